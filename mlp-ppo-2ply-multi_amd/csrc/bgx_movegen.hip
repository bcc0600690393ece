// bgx_movegen.hip — K2: legal-move generation + afterstate expansion on gfx950.
//
// Replaces get_all_possible_moves (src/backgammon/moves/generate_all_moves.py:7-90),
// handle_non_doubles / handle_doubles / add_unique_board
// (src/backgammon/moves/handle_move_types.py:7-221) and the per-move board
// application of generate_all_board_features (src/environments/env_helper.py:7-91).
//
// One job = one (board, player, dice); one wavefront per job (64-thread
// workgroups, persistent grid-stride over jobs); all job state lives in an
// LDS slice: a hash table of 64-bit {key, ordinal} words and two frontier
// lists (8 KB in tier 1, see Slice below).
//
// The reference's DFS emits the DISTINCT resulting boards in first-reach
// (lexicographic path) order and keeps the maximal-length plays. Here:
//  * every record gets an ORDINAL = its rank in that lexicographic order
//    (an exclusive prefix sum of per-parent move counts + the move index);
//  * records are deduplicated by an exact integer KEY of the resulting board:
//    LDS slot = key << 32 | ordinal, inserted with one CAS; a lane that finds
//    its key already there lowers the ordinal with one atomicMin, so each key
//    ends up holding its first-reach ordinal;
//  * parents sit one per lane and expand their children one move per
//    iteration; once a parent chunk is done, a child survives iff its ordinal
//    is the slot's ordinal, and survivors are appended in (parent, move) order.
// Non-doubles: lanes 0..15 = pass 1 (high die first), 16..31 = pass 2
//   (generate_all_moves.py:23-50); key = the canonical mover delta (removed /
//   added positions after cancelling a chained checker) + hit points.
// Doubles: up to four levels, each deduplicated on its own (equal boards have
//   equal subtrees, so the first copy carries every later first reach); key =
//   the sorted multiset of step sources in travel order. The deepest level is
//   the record set; below depth 4 a node counts only if its parent had exactly
//   one move (handle_move_types.py:117-169).
// A job whose level outgrows the LDS table is re-run by a fallback launch of
// the same code in a bigger slice, then on a global-memory workspace (exact).
#include "bgx_device.h"
#include "bgx_movegen.h"

namespace bgx {

// Tier 1 for large launches (the 2-ply replies), balanced: a workgroup of PW
// waves owns the interleaved jobs b, b + G, ... and its waves take the next
// one from an LDS counter. With a static per-wave stride the launch lasts as
// long as its unluckiest wave (67 jobs of very different cost each for the
// 344 k reply jobs of a 4,096-lane K=4 step); here a wave that drew cheap jobs
// takes more. The next job's board is loaded while the current job runs.
// Slice (4 KB per wave): a 64-word parent map, then a region that is either
// the table-mode layout (256-slot table + two 224-entry frontiers) or, for the
// table-free modes (doubles by path, non-doubles by rule: most jobs), two
// 480-entry lists laid over it. With half the round-1 8 KB slice the pool is
// bound by registers, not LDS: 16-wave workgroups, two per CU, at <= 64 VGPRs
// = 8 waves per SIMD, the hardware maximum (amdgpu_waves_per_eu). Measured on
// the 2-ply K=4 reply launch at 8,192 lanes (profiles/r2/ab_pool): 8 KB slices
// / 5 waves per SIMD 0.64 ms, 4 KB / 7 waves 0.54 ms, 4 KB / 8 waves 0.475 ms.
#ifndef BGX_REPLY_LEAF
#define BGX_REPLY_LEAF 1   // A/B builds: 0 = path doubles never stream their leaves (job_records)
#endif
#ifndef BGX_REPLY_SUBQ
#define BGX_REPLY_SUBQ 1   // A/B builds: 0 = an uncovered root's 15 jobs run on its own wave
#endif
#ifndef BGX_BND
#define BGX_BND 2          // 1 = the per-roll-round board_nd_records (A/B builds)
#endif
#ifndef BGX_REPLY_DBL_TAIL
#define BGX_REPLY_DBL_TAIL 4   // board-major doubles launch: 64ths of the rows left in per-roll items
#endif
#ifndef BGX_REPLY_WG
#define BGX_REPLY_WG 1   // A/B builds: 0 = the reply launch's waves reserve rows in per-wave chunks
#endif
#ifndef BGX_POOL_WPE
#define BGX_POOL_WPE 8
#endif
constexpr int PW = 16;                                   // waves per workgroup (two per CU)
constexpr int P_S = 256;                                 // table slots (table mode)
constexpr int P_F = 224;                                 // table-mode frontier entries
constexpr int P_PF = 480;                                // table-free list entries
constexpr int PSL = 64 * 4 + 2 * P_PF * 4;               // slice bytes (4 KB)
static_assert(P_S * 8 + 2 * P_F * 4 <= 2 * P_PF * 4, "table layout fits the region");
static_assert(PW * PSL + 16 <= 80 * 1024, "two workgroups per CU");

// IN / OUT >= 0: the input / output mode is fixed at compile time (the 2-ply
// reply launch: IN_TWOPLY, OUT_PACKED_FLAT), so the other modes' code and
// arguments are dead (fewer live scalar registers); -1: read from the arguments
template <int IN, int OUT>
__global__ __launch_bounds__(64 * PW) __attribute__((amdgpu_waves_per_eu(BGX_POOL_WPE))) void movegen_pool_kernel(
    MovegenArgs a0) {
    MovegenArgs a = a0;
    if constexpr (IN >= 0) a.in_mode = IN;
    if constexpr (OUT >= 0) a.out_mode = OUT;
    __shared__ __attribute__((aligned(16))) unsigned long long smem[PW * PSL / 8];
    __shared__ int next_job;
    const int w = (int)threadIdx.x >> 6, l = lane_id();
    uint32_t* sl = (uint32_t*)(smem + (size_t)w * (PSL / 8));
    Mem M;
    M.map = sl;
    M.tab = (unsigned long long*)(sl + 64);
    M.S = P_S;
    M.F = P_F;
    M.fa = sl + 64 + 2 * P_S;
    M.fb = M.fa + P_F;
    M.pa = sl + 64;
    M.pb = M.pa + P_PF;
    M.PF = P_PF;
    M.force_table = a.force_table;
    M.map[l] = 0u;
    const int n_jobs = uniform(job_count(a));
    // the workgroup's jobs are b, b + G, b + 2G, ... (a contiguous range would
    // hold the rolls of only ~8 root positions, whose costs are correlated);
    // its waves take them in order from the counter
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    const int nk = n_jobs > b ? (n_jobs - b + G - 1) / G : 0;
    if (threadIdx.x == 0) next_job = PW;
    __syncthreads();
    FlatCursor fc;
    int k = w;
    RawJob raw;
    if (k < nk) raw = fetch_raw(a, b + k * G);
    while (k < nk) {   // k is wave-uniform
        int kn = 0;
        if (l == 0) kn = atomicAdd(&next_job, 1);
        kn = uniform(kn);
        const int j = b + k * G;
        const JobIn in = decode_job(a, j, raw);
        if (kn < nk) raw = fetch_raw(a, b + kn * G);
        fc.left_hint = (nk - k + PW - 1) / PW;
        if (in.skip) {
            begin_emit(a, j, 0, fc);
        } else {
            const int r = a.force_tier >= 2 ? -1 : run_job<false, BGX_REPLY_LEAF != 0>(a, j, in, M, fc, a.heavy_t);
            if (r < 0 && l == 0) push_ovf(a, j);
        }
        k = kn;
    }
}

// Tier 1 of the 2-ply reply launch, board-major (IN_TWOPLY, OUT_PACKED_FLAT):
// the pool kernel's workgroups, slices and LDS job counter, but an item is a
// (candidate row, group): group 0 = the row's 15 non-doubles rolls in one
// wave (board_nd_records, one record block for the row; roots it does not
// cover run their 15 rolls as per-roll jobs), groups 1..6 = the doubles roll
// (d, d) as a per-roll job (job_records). Items are interleaved over the
// workgroups (b, b + G, ...) as the pool kernel's jobs, so the heavy doubles
// items spread. Same records, offsets and counts per job as the pool kernel
// (job order within a row's block is the DICE_ROLLS order); overflowing
// per-roll jobs go to tier 2 as before.
// DBL (the launch picks it, bgx_launch_movegen): a row's six doubles rolls in
// one item (board_dbl_emit), groups 0..1, except for the last a.dbl_tail64 / 64
// of the rows, which keep one item per doubles roll (groups 0..6): a
// workgroup's items end on the short per-roll ones, so its waves finish
// together. Not DBL: every row in per-roll items.
constexpr int REPLY_SUBQ = 1024;   // sub-queue entries per workgroup (4 KB of LDS: 2 x 68 KB per CU)
template <bool DBL>
__global__ __launch_bounds__(64 * PW) __attribute__((amdgpu_waves_per_eu(BGX_POOL_WPE))) void movegen_reply_kernel(
    MovegenArgs a0) {
    MovegenArgs a = a0;
    a.in_mode = IN_TWOPLY;
    a.out_mode = OUT_PACKED_FLAT;
    __shared__ __attribute__((aligned(16))) unsigned long long smem[PW * PSL / 8];
    __shared__ WgRows wgr;   // the workgroup's item counters and output rows (FlatCursor::wg)
    int& next_job = wgr.next;
    int& items_done = wgr.done;
    const int w = (int)threadIdx.x >> 6, l = lane_id();
    uint32_t* sl = (uint32_t*)(smem + (size_t)w * (PSL / 8));
    Mem M;
    M.map = sl;
    M.tab = (unsigned long long*)(sl + 64);
    M.S = P_S;
    M.F = P_F;
    M.fa = sl + 64 + 2 * P_S;
    M.fb = M.fa + P_F;
    M.pa = sl + 64;
    M.pb = M.pa + P_PF;
    M.PF = P_PF;
    M.force_table = a.force_table;
    M.map[l] = 0u;
    const int n_jobs = uniform(job_count(a));
    const int n_rows = (n_jobs + 20) / 21;
    // rows [0, head): items (row, 0) and (row, all doubles); rows [head, n_rows):
    // items (row, 0..6). Row-major, so a row's items run close together.
    int tail = n_rows;
    if constexpr (DBL) {
        const int t64 = a.dbl_tail64 < 0 ? 0 : a.dbl_tail64 > 64 ? 64 : a.dbl_tail64;
        tail = (int)(((long long)n_rows * t64 + 63) >> 6);
    }
    const int head = n_rows - tail, n_items = 2 * head + 7 * tail;
    // item -> (row, group); grp 1..6 with whole = the six doubles rolls at once
    auto item_row = [&](int it, int& grp, bool& whole) -> int {
        if (it < 2 * head) {
            grp = it & 1;
            whole = grp != 0;
            return it >> 1;
        }
        it -= 2 * head;
        const int q = it / 7;
        grp = it - 7 * q;
        whole = false;
        return head + q;
    };
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    const int nk = n_items > b ? (n_items - b + G - 1) / G : 0;
    // the workgroup's sub-queue: the 15 per-roll jobs of a root that
    // board_nd_records does not cover are shared by its waves (entry = job + 1,
    // 0 until the pushing wave has written it) instead of running in a row on
    // one wave (at ~13 us per job that wave ends ~190 us after the others)
    __shared__ int subq[REPLY_SUBQ];
    __shared__ int sub_res, sub_head;
    __shared__ uint32_t dcnt[DBL ? PW : 1][8];   // board_dbl_emit's per-die child counts, per wave
    for (int i = (int)threadIdx.x; i < REPLY_SUBQ; i += 64 * PW) subq[i] = 0;
    if (threadIdx.x == 0) {
        next_job = PW;
        sub_res = sub_head = items_done = 0;
        wgr.span = 0ull;
        wgr.used = 0u;
        wgr.items = nk;
    }
    __syncthreads();
    FlatCursor fc;
    if (BGX_REPLY_WG) fc.wg = &wgr;
    int k = w;
    RawJob raw;
    if (k < nk) {
        int g0;
        bool w0;
        raw = fetch_raw(a, item_row(b + k * G, g0, w0) * 21);
    }
    // one (row, roll) job as the pool kernel runs it
    auto per_roll = [&](int j, const RawJob& cur) {
        const JobIn in = decode_job(a, j, cur);
        if (in.skip) {
            begin_emit(a, j, 0, fc);
        } else {
            const int r = a.force_tier >= 2 ? -1 : run_job<false, BGX_REPLY_LEAF != 0>(a, j, in, M, fc, a.heavy_t);
            if (r < 0 && l == 0) push_ovf(a, j);
        }
    };
    auto lds_ld = [](int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // cnt per-roll jobs (job_of(q), q < cnt <= 15) onto the workgroup's sub-queue
    // when it has room (and every job index is in range), else run here
    auto share = [&](int cnt, auto job_of, bool in_range, const RawJob& cur) {
        int slot = -1;
        if (BGX_REPLY_SUBQ && l == 0 && in_range) {
            int r = lds_ld(&sub_res);
            while (r + cnt <= REPLY_SUBQ) {
                const int prev = atomicCAS(&sub_res, r, r + cnt);
                if (prev == r) {
                    slot = r;
                    break;
                }
                r = prev;
            }
        }
        slot = uniform(slot);
        if (slot >= 0) {
            if (l < cnt) __hip_atomic_store(&subq[slot + l], job_of(l) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            for (int q = 0; q < cnt; ++q) {
                const int j = job_of(q);
                if (j < n_jobs) per_roll(j, cur);
            }
        }
    };
    for (unsigned spin = 0;;) {
        // 1. a queued sub-job first (short; its root's item is done)
        int got = -1;
        if (l == 0) {
            int h = lds_ld(&sub_head);
            while (h < lds_ld(&sub_res)) {
                const int prev = atomicCAS(&sub_head, h, h + 1);
                if (prev == h) {
                    got = h;
                    break;
                }
                h = prev;
            }
        }
        got = uniform(got);
        if (got >= 0) {
            int v = 0;
            for (unsigned sp = 0; (v = uniform(lds_ld(&subq[got]))) == 0; ++sp) {   // the pusher writes it next
                if (sp >= (1u << 24)) {   // bounded
                    if (l == 0) atomicOr(a.err_flags, BGX_ERRF_WAIT_BOUND);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (v > 0) per_roll(v - 1, fetch_raw(a, v - 1));
            continue;
        }
        if (k >= nk) {
            // no items left for this wave: done once every item is done (no more
            // pushes) and the sub-queue is drained. Lane 0 reads the three counters
            // and the verdict is broadcast: the exit is wave-uniform by
            // construction, not by the hardware returning one LDS word to every
            // lane (acquire pairs with the release increment of items_done below,
            // so a drained verdict sees every push of every finished item)
            int fin = 0;
            if (l == 0)
                fin = __hip_atomic_load(&items_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= nk &&
                      lds_ld(&sub_head) >= lds_ld(&sub_res);
            if (uniform(fin)) break;
            if (++spin >= (1u << 24)) {
                if (l == 0) atomicOr(a.err_flags, BGX_ERRF_WAIT_BOUND);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        // 2. this wave's next item
        int kn = 0;
        if (l == 0) kn = atomicAdd(&next_job, 1);
        kn = uniform(kn);
        const int it = b + k * G;
        int grp;
        bool whole;
        const int row = item_row(it, grp, whole);
        const RawJob cur = raw;
        if (kn < nk) {
            int g0;
            bool w0;
            raw = fetch_raw(a, item_row(b + kn * G, g0, w0) * 21);
        }
        const int left = (nk - k + PW - 1) / PW;   // items this wave still expects
        fc.left_hint = left;
        const int j0 = row * 21;
        if (a.reply_groups && !((a.reply_groups >> grp) & 1)) {
            // tools hook: timing by group
        } else if (grp > 0 && !whole) {
            const int j = j0 + dbl_q21(grp);
            if (j < n_jobs) per_roll(j, cur);
        } else if (grp > 0) {
            if constexpr (DBL) {
                // the six doubles rolls together (path-mode roots); the rest as per-roll
                // jobs shared on the sub-queue
                const JobIn in = decode_job(a, j0, cur);   // the row's root (the dice are not used)
                uint32_t rest = 0x3Fu;
                if (in.skip && j0 + 21 <= n_jobs) {
                    for (int d = 1; d <= 6; ++d) begin_emit(a, j0 + dbl_q21(d), 0, fc);
                    rest = 0u;
                } else if (!in.skip && a.force_tier < 2 && j0 + 21 <= n_jobs) {
                    rest = board_dbl_emit<false>(a, j0, in, M, fc, dcnt[w]);
                }
                if (rest)
                    share(__popc(rest), [&](int q) { return j0 + dbl_q21(select_bit((uint32_t)rest, q) + 1); },
                          j0 + 21 <= n_jobs, cur);
            }
        } else {
            const JobIn in = decode_job(a, j0 + 1, cur);   // the row's root (the dice are not used)
            int n = -1, rc = 0;
            if (!in.skip && !a.force_table && a.force_tier < 2 && j0 + 21 <= n_jobs && !(a.reply_groups & 0x100))
                n = BGX_BND == 2 ? board_nd_records2<P_PF>(in.R, M.map, M.pa, M.pb, rc)
                                 : board_nd_records<P_PF>(in.R, M.map, M.pa, rc);
            if (n < 0 && (a.reply_groups & 0x80)) n = -2;   // tools hook: leave uncovered roots out
            if (n >= 0) {
                // the row's records in one block; job q's records at its prefix
                const int base = reserve_flat(a, n, fc, 24 * 15 * left);
                const int pre = wave_incl_scan(rc) - rc;
                if (l < ND_ROLLS) {
                    const int j = j0 + nd_roll_q21(l);
                    if (BGX_DBL_GUARD && (j >= n_jobs || (base >= 0 && base + pre + rc > a.flat_cap))) {
                        atomicOr(a.err_flags, 0x1000u);
                    } else {
                        a.job_off[j] = base < 0 ? 0 : base + pre;
                        a.job_cnt[j] = base < 0 ? 0 : rc;
                    }
                }
                if (base >= 0) {
                    for (int i = l; i < n; i += 64) {
                        const uint32_t e = M.pa[i];
                        emit_one(a, j0, in.R, nd_board(in.R, e), i, base);   // (j0: the row's root slot)
                    }
                }
                wave_sync();   // the list is read before the next item reuses the slice
            } else if (n == -1) {
                // not covered (bear-off range, or a test hook): its 15 rolls go to the
                // sub-queue when it has room, else run here. (A balanced pool launch
                // over all such jobs measured slower: its chunk reservations left
                // 12 % more gap rows for the reply MLP, profiles/round4/reply/.)
                int slot = -1;
                if (BGX_REPLY_SUBQ && l == 0 && j0 + 21 <= n_jobs) {
                    int r = lds_ld(&sub_res);
                    while (r + ND_ROLLS <= REPLY_SUBQ) {
                        const int prev = atomicCAS(&sub_res, r, r + ND_ROLLS);
                        if (prev == r) {
                            slot = r;
                            break;
                        }
                        r = prev;
                    }
                }
                slot = uniform(slot);
                if (slot >= 0) {
                    if (l < ND_ROLLS) __hip_atomic_store(&subq[slot + l], j0 + nd_roll_q21(l) + 1, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    for (int q = 0; q < ND_ROLLS; ++q) {
                        const int j = j0 + nd_roll_q21(q);
                        if (j < n_jobs) per_roll(j, cur);
                    }
                }
            }
        }
        // release: the item's sub-queue stores (lanes < 15, above) are ordered
        // before the count that lets waves leave (the wave's LDS stores are
        // complete at the fence this emits)
        wave_sync();
        if (l == 0) __hip_atomic_fetch_add(&items_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        k = kn;
    }
}

// Tier 1 for launches with few jobs (the 1-ply step, the first 2-ply launch):
// 16-wave blocks, one job per wave per window. The block reserves its rows of
// the flat output with ONE atomic (a same-address global atomic costs ~11 ns
// in series: one per job would serialise 4,096 jobs for ~45 us) and each
// wave writes its records at its prefix within the block.
// Slices as the pool kernel's (4 KB): two blocks per CU; IN / OUT as the pool
// kernel's (the engine's root launch: IN_PACKED, OUT_PACKED_FLAT).
template <int IN, int OUT>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(8))) void movegen_few_kernel(MovegenArgs a0) {
    MovegenArgs a = a0;
    if constexpr (IN >= 0) a.in_mode = IN;
    if constexpr (OUT >= 0) a.out_mode = OUT;
    __shared__ __attribute__((aligned(16))) unsigned long long smem[BW * PSL / 8];
    __shared__ uint32_t wcnt[BW];
    __shared__ int base_s;
    const int w = (int)threadIdx.x >> 6, l = lane_id();
    const int n_jobs = uniform(job_count(a));
    uint32_t* sl = (uint32_t*)(smem + (size_t)w * (PSL / 8));
    Mem M;
    M.map = sl;
    M.tab = (unsigned long long*)(sl + 64);
    M.S = P_S;
    M.F = P_F;
    M.fa = sl + 64 + 2 * P_S;
    M.fb = M.fa + P_F;
    M.pa = sl + 64;
    M.pb = M.pa + P_PF;
    M.PF = P_PF;
    M.force_table = a.force_table;
    M.map[l] = 0u;
    for (int win = (int)blockIdx.x; win * BW < n_jobs; win += (int)gridDim.x) {
        const int j = win * BW + w;
        int nf = 0;
        bool emit = false;
        uint32_t* fin = nullptr;
        JobIn in;
        if (j < n_jobs) {
            in = fetch_job(a, j);
            if (in.skip) {
                emit = true;
            } else {
                const int r = a.force_tier >= 2 ? -1 : job_records<false>(in, M, fin, a.heavy_t);
                if (r < 0) {
                    if (l == 0) push_ovf(a, j);   // overflow or heavy doubles: tier 2 owns the job
                } else {
                    emit = true;
                    nf = r;
                }
            }
        }
        if (l == 0) wcnt[w] = emit ? (uint32_t)nf : 0u;
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int k = 0; k < BW; ++k) {
            const int c = (int)wcnt[k];
            before += k < w ? c : 0;
            total += c;
        }
        if (a.out_mode == OUT_PACKED_FLAT) {
            if (threadIdx.x == 0) {
                int base = total ? (int)atomicAdd(a.flat_count, (unsigned)total) : 0;
                if (base + total > a.flat_cap) {
                    atomicOr(a.err_flags, BGX_ERRF_FLAT_OVERFLOW);
                    base = -1;
                }
                base_s = base;
            }
            __syncthreads();
            const int base = base_s;
            if (emit) {
                if (l == 0) {
                    a.job_off[j] = base < 0 ? 0 : base + before;
                    a.job_cnt[j] = base < 0 ? 0 : nf;
                }
                if (base >= 0 && nf) emit_records<false>(a, j, in, fin, nf, base + before);
            }
        } else if (emit) {
            if (l == 0) a.out_count[j] = nf;
            if (nf) emit_records<false>(a, j, in, fin, nf, 0);
        }
        __syncthreads();   // the slices are reused by the next window
    }
}

// Tier 2, one 16-wave block per listed job: doubles are expanded by the
// whole block (coop_doubles); a non-doubles job runs in wave 0 in a 32 KB
// slice. A job that still does not fit (tier 3) runs in wave 0 over the
// block's global-memory workspace (same code, exact).
__global__ __launch_bounds__(NTH) void movegen_block_kernel(MovegenArgs a) {
    const int n = (int)__hip_atomic_load(a.ovf_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int cnt = n < a.ovf_cap ? n : a.ovf_cap;
    if ((int)blockIdx.x >= cnt) return;
    __shared__ __attribute__((aligned(16))) unsigned long long smem[sizeof(CoopLds) / 8];
    __shared__ uint32_t emit_s;
    CoopLds& C = *(CoopLds*)smem;
    const int w = (int)threadIdx.x >> 6, l = lane_id();
    FlatCursor fc;
    // tier 3, wave 0 only
    auto run_global = [&](int j, const JobIn& in) {
        uint32_t* base = a.ws_global + (size_t)blockIdx.x * a.ws_words_per_wave;
        Mem G;
        const int S = a.ws_slots;
        G.tab = (unsigned long long*)base;
        G.fa = base + 2 * S;
        G.fb = base + 3 * S;
        G.map = base + 4 * S;
        G.S = S;
        G.F = S;
        G.force_table = a.force_table;
        st32<true>(G.map + l, 0u);
        sync<true>();
        if (run_job<true>(a, j, in, G, fc) < 0 && l == 0) atomicOr(a.err_flags, BGX_ERRF_FALLBACK_OVERFLOW);
    };
    for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
        const int j = a.ovf_list[t];
        const JobIn in = fetch_job(a, j);
        if (in.d0 != in.d1 || a.force_tier >= 3) {
            if (w == 0) {
                static_assert(Slice<S_T2>::bytes <= sizeof(CoopLds), "slice fits");
                Mem M = lds_mem<S_T2>(smem);
                M.force_table = a.force_table;
                const int r = a.force_tier >= 3 ? -1 : run_job<false>(a, j, in, M, fc);
                if (r < 0) run_global(j, in);
            }
            __syncthreads();
            continue;
        }
        uint32_t* fin = nullptr;
        const int nfin = coop_doubles(in, C, fin, a.force_table != 0);
        if (nfin < 0) {
            if (w == 0) run_global(j, in);
            __syncthreads();
            continue;
        }
        if (w == 0) {
            const int base = begin_emit(a, j, nfin, fc);
            if (l == 0) emit_s = (uint32_t)base;
        }
        __syncthreads();
        const int base = (int)emit_s;
        if (base >= 0) {
            for (int i = (int)threadIdx.x; i < nfin; i += NTH) {
                const uint32_t e = fin[i];
                emit_one(a, j, in.R,
                         (e & PATHF) ? path_board(in.R, e & KEYMASK, in.d0) : rebuild(in.R, e & KEYMASK, in.d0),
                         i, base);
            }
        }
        __syncthreads();
    }
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_movegen(const bgx::MovegenArgs* args, hipStream_t stream) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    bgx::MovegenArgs a = *args;
    if (a.n_jobs <= 0 && !a.n_jobs_dev) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!a.ovf_zeroed) {
        e = hipMemsetAsync(a.ovf_count, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
    }
    // resident blocks per CU of each kernel (LDS, registers, 32 waves)
    static int per_cub = 0, per_cuf = 0, per_cup = 0;
    if (!per_cub) {
        auto occ = [](int& n, const void* k, int threads, int dflt) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, threads, 0) != hipSuccess || n <= 0) n = dflt;
        };
        occ(per_cup, (const void*)bgx::movegen_pool_kernel<-1, -1>, 64 * bgx::PW, 2);
        occ(per_cub, (const void*)bgx::movegen_block_kernel, bgx::NTH, 1);
        occ(per_cuf, (const void*)bgx::movegen_few_kernel<-1, -1>, bgx::NTH, 1);
    }
    // test hooks (parity cross-checks; three getenv per launch, next to a
    // kernel launch's cost): BGX_MG_TEST_TIER=2/3 routes every job to tier 2 / 3;
    // BGX_MG_TEST_TABLE=1 sends every job down the hash-table path; BGX_MG_FEW=0/1
    // forces the tier-1 kernel choice below (the two kernels give identical rows)
    const char* ev = getenv("BGX_MG_TEST_TIER");
    const int test_tier = ev ? atoi(ev) : 0;
    ev = getenv("BGX_MG_TEST_TABLE");
    const int test_table = ev ? atoi(ev) : 0;
    ev = getenv("BGX_MG_FEW");
    const int fewm = ev ? atoi(ev) : -1;
    a.force_tier = test_tier;
    a.force_table = test_table;
    ev = getenv("BGX_REPLY_GROUPS");
    a.reply_groups = ev ? (int)strtol(ev, nullptr, 0) : 0;
    // doubles run table-free in tier 1 (the block-cooperative hand-off of heavy
    // doubles measured slower since then: DESIGN.md §4)
    a.heavy_t = 0x7FFFFFFF;
    // latency-bound launches (at most 4 windows of 16 jobs per CU, host-known
    // count): tier 1 in 16-wave blocks with one flat-row atomic per block;
    // larger launches: the balanced pool kernel
    const bool few_jobs = !a.n_jobs_dev && a.n_jobs <= n_cu * per_cuf * bgx::BW * 4;
    if (fewm == 1 || (fewm < 0 && few_jobs)) {
        int blocks = a.n_jobs_dev ? n_cu * per_cuf : (a.n_jobs + bgx::BW - 1) / bgx::BW;
        if (blocks > n_cu * per_cuf) blocks = n_cu * per_cuf;
        if (a.in_mode == bgx::IN_PACKED && a.out_mode == bgx::OUT_PACKED_FLAT)
            hipLaunchKernelGGL((bgx::movegen_few_kernel<bgx::IN_PACKED, bgx::OUT_PACKED_FLAT>), dim3(blocks),
                               dim3(bgx::NTH), 0, stream, a);
        else
            hipLaunchKernelGGL((bgx::movegen_few_kernel<-1, -1>), dim3(blocks), dim3(bgx::NTH), 0, stream, a);
    } else {
        int blocks = n_cu * per_cup;
        const int need = (a.n_jobs + bgx::PW - 1) / bgx::PW;
        if (!a.n_jobs_dev && need < blocks) blocks = need;
        // BGX_REPLY_BM=0: the 2-ply replies as per-(row, roll) jobs (the A/B and
        // cross-check arm; identical records)
        ev = getenv("BGX_REPLY_BM");
        const bool bm = !ev || atoi(ev) != 0;
        if (a.in_mode == bgx::IN_TWOPLY && a.out_mode == bgx::OUT_PACKED_FLAT && bm) {
            // the doubles rolls of a row: one item (board_dbl_emit), except for the
            // last BGX_REPLY_DBL_TAIL / 64 of the rows, whose six rolls are six
            // items, so a workgroup ends on short items. K = 4 at 8,192 lanes (32,768
            // rows over 512 workgroups), per-wave row chunks: 1.590 ms per step with
            // per-roll items only, 1.667 with none of them, 1.532-1.536 with 10-24 /
            // 64 (tools/runs/README.md r5_l, r5_m); with the workgroup row chunks the
            // best tails are smaller: 2-4 / 64 1.405-1.411 ms, 12 / 64 1.419-1.424
            // (r5_s, r5_t); K = all within noise (7.69-7.80 ms for 0-12).
            // BGX_REPLY_DBL=0: per-roll doubles items only (tests, A/B).
            ev = getenv("BGX_REPLY_DBL");
            const bool dbl = !ev || atoi(ev) != 0;
            ev = getenv("BGX_REPLY_DBL_TAIL");
            a.dbl_tail64 = ev ? atoi(ev) : BGX_REPLY_DBL_TAIL;
            int rb = n_cu * per_cup;
            const int need_r = ((a.n_jobs + 20) / 21 * 7 + bgx::PW - 1) / bgx::PW;   // at most 7 items per row
            if (!a.n_jobs_dev && need_r < rb) rb = need_r;
            if (dbl)
                hipLaunchKernelGGL(bgx::movegen_reply_kernel<true>, dim3(rb), dim3(64 * bgx::PW), 0, stream, a);
            else
                hipLaunchKernelGGL(bgx::movegen_reply_kernel<false>, dim3(rb), dim3(64 * bgx::PW), 0, stream, a);
        } else if (a.in_mode == bgx::IN_TWOPLY && a.out_mode == bgx::OUT_PACKED_FLAT)
            hipLaunchKernelGGL((bgx::movegen_pool_kernel<bgx::IN_TWOPLY, bgx::OUT_PACKED_FLAT>), dim3(blocks),
                               dim3(64 * bgx::PW), 0, stream, a);
        else
            hipLaunchKernelGGL((bgx::movegen_pool_kernel<-1, -1>), dim3(blocks), dim3(64 * bgx::PW), 0, stream, a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // tier 2 (+ tier 3 in the same block): one block per CU, at most one per workspace slice
    int bblocks = n_cu * per_cub;
    if (bblocks > a.ws_waves) bblocks = a.ws_waves;
    hipLaunchKernelGGL(bgx::movegen_block_kernel, dim3(bblocks), dim3(bgx::NTH), 0, stream, a);
    return hipGetLastError();
}
