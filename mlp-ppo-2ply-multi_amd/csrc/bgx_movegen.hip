// bgx_movegen.hip — K2: legal-move generation + afterstate expansion on gfx950.
//
// Replaces get_all_possible_moves (src/backgammon/moves/generate_all_moves.py:7-90),
// handle_non_doubles / handle_doubles / add_unique_board
// (src/backgammon/moves/handle_move_types.py:7-221) and the per-move board
// application of generate_all_board_features (src/environments/env_helper.py:7-91).
//
// One job = one (board, player, dice). One wavefront per job; four independent
// jobs per 256-thread workgroup; all job state in that wave's LDS slice.
//
// The reference DFS records the DISTINCT resulting boards in first-reach
// (lexicographic path) order and keeps the maximal-length plays. The wave
// reproduces that order level-synchronously:
//  * non-doubles: the <=15 first sub-moves of each pass sit on lanes 0..31
//    (pass 1 = high die first on lanes 0..15, pass 2 on 16..31); the 2-move
//    records are enumerated in (pass, i, j) order by a wave prefix sum, then
//    deduplicated keeping the smallest ordinal (a per-slot atomicMin in an LDS
//    hash table keyed by the exact 128-bit result board). The pass-2 skip
//    (generate_all_moves.py:40-50) and the singles fallback
//    (handle_move_types.py:70-81) are applied from wave ballots.
//  * doubles: levels 1..4 are expanded breadth-first; each level's children are
//    generated in (parent order, move order) = DFS order and deduplicated
//    against that level only (two nodes with the same board have identical
//    subtrees, so keeping the first keeps every later first-reach position).
//    A node is the sorted multiset of its step sources in travel order — an
//    exact 20-bit key of the board for a fixed root and die. The deepest
//    non-empty level holds the records; below depth 4 a node is a record only
//    when its parent had exactly one move (handle_move_types.py:117-169).
// Jobs whose doubles frontier outgrows the LDS slice are re-run by a fallback
// launch of the same code over a global-memory workspace (exact, just slower).
#include "bgx_device.h"
#include "bgx_kernels.h"

namespace bgx {

constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr uint32_t KEY_EMPTY4 = 0xFFFFFu;   // four empty 5-bit fields
constexpr uint32_t KEYMASK = 0xFFFFFu;

// LDS slice per wave (uint32 words)
constexpr int S_D = 1024;   // doubles hash slots
constexpr int F_D = 1024;   // doubles frontier capacity
constexpr int S_N = 512;    // non-doubles hash slots (<= 450 records)
constexpr int WAVE_WORDS = 5 * 1024;   // tkey, tmin, fa, fb, pre  (20 KB)

struct Mem {
    uint32_t* tkey;   // [S]      doubles keys
    uint32_t* tmin;   // [S]      min ordinal per slot (EMPTY = free)
    uint32_t* fa;     // [F]
    uint32_t* fb;     // [F]
    uint32_t* pre;    // [F]
    uint4* tkey4;     // [S_N]    non-doubles keys (overlays fa/fb)
    uint32_t* surv;   // [S_N]    non-doubles survivor slots (overlays pre)
    int S, F;
};

// memory-kind dependent accessors: LDS (wavefront scope) or global (agent scope)
template <bool G> BGX_DEV uint32_t ld(const uint32_t* p) {
    if constexpr (G) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV void st(uint32_t* p, uint32_t v) {
    if constexpr (G) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV uint32_t cas(uint32_t* p, uint32_t cmp, uint32_t v) {
    if constexpr (G) {
        __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    return cmp;
}
template <bool G> BGX_DEV void amin(uint32_t* p, uint32_t v) {
    if constexpr (G) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV void sync() {
    if constexpr (G) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else {
        wave_sync();
    }
}

template <bool G> BGX_DEV void clear(uint32_t* p, int n) {
    for (int i = lane_id(); i < n; i += 64) st<G>(p + i, EMPTY);
    sync<G>();
}

BGX_DEV uint32_t hash32(uint32_t k) { return k * 0x9E3779B1u; }
BGX_DEV uint32_t hash128(const Node& n) {
    uint32_t h = n.m0 * 0x9E3779B1u;
    h ^= (n.m1 + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= (n.m2 + 0x165667B1u) * 0xC2B2AE3Du;
    h ^= (n.x + 0x27D4EB2Fu) * 0x9E3779B1u;
    return h ^ (h >> 15);
}

// Deduplicate one chunk (<= 64 records, ordinals increasing across chunks).
// Returns true on lanes whose record is the first occurrence of its key.
template <bool G>
BGX_DEV bool dedup_u32(const Mem& M, bool active, uint32_t key, uint32_t ord) {
    const uint32_t mask = (uint32_t)M.S - 1u;
    const int shift = 32 - __builtin_ctz((uint32_t)M.S);
    uint32_t slot = hash32(key) >> shift;
    bool pending = active;
    uint32_t my = 0;
    while (ballot(pending)) {
        if (pending && ld<G>(M.tmin + slot) == EMPTY) {
            if (cas<G>(M.tmin + slot, EMPTY, ord) == EMPTY) st<G>(M.tkey + slot, key);
        }
        sync<G>();
        if (pending) {
            if (ld<G>(M.tkey + slot) == key) {
                amin<G>(M.tmin + slot, ord);
                my = slot;
                pending = false;
            } else {
                slot = (slot + 1u) & mask;
            }
        }
        sync<G>();
    }
    return active && ld<G>(M.tmin + my) == ord;
}

template <bool G>
BGX_DEV bool dedup_128(const Mem& M, bool active, const Node& key, uint32_t ord, uint32_t& myslot) {
    const uint32_t mask = S_N - 1u;
    uint32_t slot = (hash128(key) >> 23) & mask;
    bool pending = active;
    uint32_t my = 0;
    while (ballot(pending)) {
        if (pending && ld<G>(M.tmin + slot) == EMPTY) {
            if (cas<G>(M.tmin + slot, EMPTY, ord) == EMPTY) {
                uint32_t* k = (uint32_t*)(M.tkey4 + slot);
                st<G>(k + 0, key.m0); st<G>(k + 1, key.m1); st<G>(k + 2, key.m2); st<G>(k + 3, key.x);
            }
        }
        sync<G>();
        if (pending) {
            const uint32_t* k = (const uint32_t*)(M.tkey4 + slot);
            bool eq = ld<G>(k + 0) == key.m0 && ld<G>(k + 1) == key.m1 && ld<G>(k + 2) == key.m2 &&
                      ld<G>(k + 3) == key.x;
            if (eq) {
                amin<G>(M.tmin + slot, ord);
                my = slot;
                pending = false;
            } else {
                slot = (slot + 1u) & mask;
            }
        }
        sync<G>();
    }
    myslot = my;
    return active && ld<G>(M.tmin + my) == ord;
}

// relative source (travel order): 0 = BAR, then points from the mover's start
BGX_DEV uint32_t rel_of(int s, int player) {
    if (s == 24) return 0u;
    return player == 0 ? (uint32_t)(s + 1) : (uint32_t)(24 - s);
}
BGX_DEV int abs_of(uint32_t rel, int player) {
    if (rel == 0u) return 24;
    return player == 0 ? (int)rel - 1 : 24 - (int)rel;
}
BGX_DEV uint32_t key_insert(uint32_t key, uint32_t rel) {
    uint32_t out = 0;
    int o = 0;
    bool placed = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t f = (key >> (5 * i)) & 31u;
        if (!placed && rel <= f) { out |= rel << (5 * o); ++o; placed = true; }
        if (o < 4) { out |= f << (5 * o); ++o; }
    }
    return out;
}
BGX_DEV Node rebuild(const Root& R, uint32_t key, int d) {
    Node n = root_node(R);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t f = (key >> (5 * i)) & 31u;
        if (f != 31u) n = apply_move(R, n, abs_of(f, R.player), d);
    }
    return n;
}

// ------------------------------------------------------------------ job I/O
struct JobIn { Root R; int d0, d1; bool skip; };

BGX_DEV JobIn fetch_job(const MovegenArgs& a, int j) {
    JobIn in;
    uint32_t w[8];
    int player = 0;
    in.skip = false;
    if (a.in_mode == IN_U8) {
        const uint32_t* b = (const uint32_t*)(a.in_u8 + (size_t)j * 52);
        uint32_t t[13];
#pragma unroll
        for (int i = 0; i < 13; ++i) t[i] = b[i];
        player = a.in_player[j];
        u8_to_packed(t, 0, w);
        in.d0 = a.in_dice[2 * j];
        in.d1 = a.in_dice[2 * j + 1];
    } else if (a.in_mode == IN_PACKED) {
        const uint4* p = (const uint4*)(a.in_packed + (size_t)j * 8);
        uint4 x = p[0], y = p[1];
        w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
        player = a.in_player[j];
        in.d0 = a.in_dice[2 * j];
        in.d1 = a.in_dice[2 * j + 1];
    } else {  // IN_TWOPLY: job = row * 21 + roll; board = candidate row; player = opponent
        int row = j / 21, roll = j - 21 * (j / 21);
        int src = a.in_rows ? a.in_rows[row] : a.in_row_base + row;
        if (src < 0) {
            in.skip = true;
            src = 0;
        }
        const uint4* p = (const uint4*)(a.in_packed + (size_t)src * 8);
        uint4 x = p[0], y = p[1];
        w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
        player = 1 - (int)((w[6] >> 16) & 1u);
        // DICE_ROLLS (two_ply.py:10-32): (1,1),(1,2)..(1,6),(2,2)..(6,6)
        int a0 = 1, r = roll;
        while (r >= 7 - a0) { r -= 7 - a0; ++a0; }
        in.d0 = a0;
        in.d1 = a0 + r;
    }
    // wave-uniform root (player chosen by selects, no dynamic register indexing)
    uint32_t s6 = w[6];
    Root& R = in.R;
    bool p2 = player != 0;
    R.m0 = p2 ? w[3] : w[0]; R.m1 = p2 ? w[4] : w[1]; R.m2 = p2 ? w[5] : w[2];
    R.o0 = p2 ? w[0] : w[3]; R.o1 = p2 ? w[1] : w[4]; R.o2 = p2 ? w[2] : w[5];
    uint32_t b0 = s6 & 15u, b1 = (s6 >> 4) & 15u, f0 = (s6 >> 8) & 15u, f1 = (s6 >> 12) & 15u;
    R.bar = p2 ? b1 : b0; R.obar = p2 ? b0 : b1;
    R.off = p2 ? f1 : f0; R.ooff = p2 ? f0 : f1;
    R.block = ge2_24(R.o0, R.o1, R.o2);
    R.blot = occ24(R.o0, R.o1, R.o2) & ~R.block;
    R.player = player;
    return in;
}

// write one record (lane-local) at output position k of job j
BGX_DEV void emit_one(const MovegenArgs& a, int j, const Root& R, const Node& n, int k, int base) {
    uint32_t w[8];
    node_to_packed(R, n, (uint32_t)R.player, w);
    if (a.out_mode == OUT_U8) {
        if (k >= a.cap) return;
        uint32_t o[13];
        packed_to_u8(w, o);
        uint32_t* dst = (uint32_t*)(a.out_u8 + ((size_t)j * a.cap + k) * 52);
#pragma unroll
        for (int i = 0; i < 13; ++i) dst[i] = o[i];
    } else if (a.out_mode == OUT_PACKED_SLOT) {
        if (k >= a.cap) return;
        uint4* dst = (uint4*)(a.out_packed + ((size_t)j * a.cap + k) * 8);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {  // OUT_PACKED_FLAT
        uint4* dst = (uint4*)(a.out_packed + ((size_t)base + k) * 8);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

// reserve output space once the job's record count is known; returns base
BGX_DEV int begin_emit(const MovegenArgs& a, int j, int n) {
    int base = 0;
    if (a.out_mode == OUT_PACKED_FLAT) {
        if (lane_id() == 0) {
            base = (int)atomicAdd(a.flat_count, (unsigned)n);
            if (base + n > a.flat_cap) {
                atomicOr(a.err_flags, BGX_ERRF_FLAT_OVERFLOW);
                base = -1;
            }
        }
        base = uniform(base);
        if (lane_id() == 0) {
            a.job_off[j] = base < 0 ? 0 : base;
            a.job_cnt[j] = base < 0 ? 0 : n;
        }
    } else if (lane_id() == 0) {
        a.out_count[j] = n;
    }
    return base;
}

// ------------------------------------------------------------------ the job
// returns the record count, or -1 when the LDS slice overflowed (doubles only)
template <bool G>
BGX_DEV int run_job(const MovegenArgs& a, int j, const JobIn& in, const Mem& M) {
    const Root& R = in.R;
    const int l = lane_id();
    const Node root = root_node(R);

    if (in.d0 != in.d1) {
        // ------------------------------------------------ non-doubles
        const int H = in.d0 > in.d1 ? in.d0 : in.d1, L = in.d0 > in.d1 ? in.d1 : in.d0;
        const uint32_t okH = ok_mask(R.block, H, R.player), okL = ok_mask(R.block, L, R.player);
        const Moves mH = node_moves(R, root, H, okH), mL = node_moves(R, root, L, okL);
        const int pass = (l >> 4) & 1, k = l & 15;
        const bool in32 = l < 32;
        const int dA = pass ? L : H, dB = pass ? H : L;
        const uint32_t okB = pass ? okH : okL;
        const bool v1 = in32 && k < (pass ? mL.n : mH.n);
        Node child = root;
        int c = 0;
        if (v1) {
            child = apply_move(R, root, move_source(pass ? mL : mH, k), dA);
            c = node_moves(R, child, dB, okB).n;
        }
        const bool two1 = ballot(in32 && pass == 0 && c > 0) != 0ull;
        const bool two2 = ballot(in32 && pass == 1 && c > 0) != 0ull;
        const int nH = mH.n, nL = mL.n;
        clear<G>(M.tmin, S_N);
        int nsurv = 0;
        if (two1 || (nH != 1 && two2)) {
            // 2-move records in (pass, i, j) order (handle_non_doubles 43-68, both passes)
            const int cc = in32 ? c : 0;
            const int incl = wave_incl_scan(cc);
            const int excl = incl - cc;
            const int T = __shfl(incl, 63, 64);
            for (int b = 0; b < T; b += 64) {
                const int r = b + l;
                const bool act = r < T;
                int p = 0;
#pragma unroll
                for (int step = 16; step >= 1; step >>= 1) {
                    int q = p + step;
                    int e = __shfl(excl, q & 31, 64);
                    if (q < 32 && e <= r) p = q;
                }
                const int ep = __shfl(excl, p, 64);
                Node ch = root;
                if (act) {
                    const int ppass = p >> 4, pk = p & 15;
                    const int pA = ppass ? L : H, pB = ppass ? H : L;
                    const Node pc = apply_move(R, root, move_source(ppass ? mL : mH, pk), pA);
                    const Moves pm = node_moves(R, pc, pB, ppass ? okH : okL);
                    ch = apply_move(R, pc, move_source(pm, r - ep), pB);
                }
                uint32_t slot;
                const bool sv = dedup_128<G>(M, act, ch, (uint32_t)r, slot);
                const uint64_t bm = ballot(sv);
                if (sv) st<G>(M.surv + nsurv + mask_prefix(bm), slot);
                nsurv += __popcll(bm);
                sync<G>();
            }
        } else {
            // singles: high-die singles, then (unless skipped) low-die singles
            // (handle_non_doubles 70-81; generate_all_moves.py:40-50)
            const int nL2 = (nH == 1) ? 0 : nL;
            const bool act = v1 && (pass == 0 || k < nL2);
            const uint32_t ord = pass == 0 ? (uint32_t)k : (uint32_t)(nH + k);
            uint32_t slot;
            const bool sv = dedup_128<G>(M, act, child, ord, slot);
            const uint64_t bm = ballot(sv);
            if (sv) st<G>(M.surv + mask_prefix(bm), slot);
            nsurv = __popcll(bm);
            sync<G>();
        }
        const int base = begin_emit(a, j, nsurv);
        if (base < 0) return nsurv;
        for (int b = 0; b < nsurv; b += 64) {
            const int i = b + l;
            if (i < nsurv) {
                const uint32_t* kk = (const uint32_t*)(M.tkey4 + ld<G>(M.surv + i));
                Node n = {ld<G>(kk), ld<G>(kk + 1), ld<G>(kk + 2), ld<G>(kk + 3)};
                emit_one(a, j, R, n, i, base);
            }
        }
        return nsurv;
    }

    // ---------------------------------------------------- doubles
    const int d = in.d0;
    const uint32_t okd = ok_mask(R.block, d, R.player);
    uint32_t* fa = M.fa;
    uint32_t* fb = M.fb;
    if (l == 0) st<G>(fa, KEY_EMPTY4);
    sync<G>();
    int n = 1, level = 0;
    while (level < 4) {
        // children per frontier node -> exclusive prefix in pre[]
        int T = 0;
        for (int b = 0; b < n; b += 64) {
            const int i = b + l;
            int c = 0;
            if (i < n) c = node_moves(R, rebuild(R, ld<G>(fa + i) & KEYMASK, d), d, okd).n;
            const int incl = wave_incl_scan(c);
            if (i < n) st<G>(M.pre + i, (uint32_t)(T + incl - c));
            T += __shfl(incl, 63, 64);
        }
        sync<G>();
        if (T == 0) break;
        clear<G>(M.tmin, M.S);
        int nn = 0;
        for (int b = 0; b < T; b += 64) {
            if (nn + 64 > M.S - 1) return -1;   // LDS slice too small: fallback
            const int r = b + l;
            const bool act = r < T;
            uint32_t key = 0;
            bool flag = false;
            if (act) {
                // parent = largest p with pre[p] <= r
                int lo = 0, hi = n - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((int)ld<G>(M.pre + mid) <= r) lo = mid; else hi = mid - 1;
                }
                const uint32_t pkey = ld<G>(fa + lo) & KEYMASK;
                const Moves pm = node_moves(R, rebuild(R, pkey, d), d, okd);
                const int s = move_source(pm, r - (int)ld<G>(M.pre + lo));
                key = key_insert(pkey, rel_of(s, R.player));
                flag = pm.n == 1;
            }
            const bool sv = dedup_u32<G>(M, act, key, (uint32_t)r);
            const uint64_t bm = ballot(sv);
            if (sv) st<G>(fb + nn + mask_prefix(bm), key | (flag ? 0x80000000u : 0u));
            nn += __popcll(bm);
            sync<G>();
        }
        uint32_t* t = fa; fa = fb; fb = t;
        n = nn;
        ++level;
    }
    // records: the deepest level; below depth 4 only nodes whose parent had one move
    int total = 0;
    if (level > 0) {
        for (int b = 0; b < n; b += 64) {
            const int i = b + l;
            const bool rec = i < n && (level == 4 || (ld<G>(fa + i) & 0x80000000u));
            total += __popcll(ballot(rec));
        }
    }
    const int base = begin_emit(a, j, total);
    if (base < 0 || level == 0) return total;
    int o = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + l;
        const uint32_t e = i < n ? ld<G>(fa + i) : 0u;
        const bool rec = i < n && (level == 4 || (e & 0x80000000u));
        const uint64_t bm = ballot(rec);
        if (rec) emit_one(a, j, R, rebuild(R, e & KEYMASK, d), o + mask_prefix(bm), base);
        o += __popcll(bm);
    }
    return total;
}

// ------------------------------------------------------------------ kernels
BGX_DEV int job_count(const MovegenArgs& a) {
    int n = a.n_jobs;
    if (a.n_jobs_dev) n += (int)(*a.n_jobs_dev) * a.jobs_per_dev_unit;
    return n;
}

// Persistent: each wave walks jobs j = wave_id, wave_id + total_waves, ...
__global__ __launch_bounds__(256) void movegen_lds_kernel(MovegenArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t smem[4 * WAVE_WORDS];
    const int wave = threadIdx.x >> 6;
    uint32_t* base = smem + wave * WAVE_WORDS;
    Mem M;
    M.tkey = base;
    M.tmin = base + 1024;
    M.fa = base + 2048;
    M.fb = base + 3072;
    M.pre = base + 4096;
    M.tkey4 = (uint4*)(base + 2048);   // 512 x 16 B = fa + fb
    M.surv = base + 4096;
    M.S = S_D;
    M.F = F_D;
    const int n_jobs = uniform(job_count(a));
    for (int j = uniform((int)blockIdx.x * 4 + wave); j < n_jobs; j += (int)gridDim.x * 4) {
        const JobIn in = fetch_job(a, j);
        if (in.skip) {
            begin_emit(a, j, 0);
            continue;
        }
        const int r = run_job<false>(a, j, in, M);
        if (r < 0 && lane_id() == 0) {
            unsigned slot = atomicAdd(a.ovf_count, 1u);
            if ((int)slot < a.ovf_cap) a.ovf_list[slot] = j;
            else atomicOr(a.err_flags, BGX_ERRF_OVF_LIST);
        }
    }
}

// Fallback for overflowed jobs: same code over a per-wave global workspace.
__global__ __launch_bounds__(64) void movegen_global_kernel(MovegenArgs a) {
    const int n = (int)__hip_atomic_load(a.ovf_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int cnt = n < a.ovf_cap ? n : a.ovf_cap;
    uint32_t* base = a.ws_global + (size_t)blockIdx.x * a.ws_words_per_wave;
    Mem M;
    const int S = a.ws_slots;
    M.tkey = base;
    M.tmin = base + S;
    M.fa = base + 2 * S;
    M.fb = base + 3 * S;
    M.pre = base + 4 * S;
    M.tkey4 = (uint4*)(base + 2 * S);
    M.surv = base + 4 * S;
    M.S = S;
    M.F = S;
    for (int t = blockIdx.x; t < cnt; t += gridDim.x) {
        const int j = uniform(a.ovf_list[t]);
        const JobIn in = fetch_job(a, j);
        const int r = run_job<true>(a, j, in, M);
        if (r < 0 && lane_id() == 0) atomicOr(a.err_flags, BGX_ERRF_FALLBACK_OVERFLOW);
    }
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_movegen(const bgx::MovegenArgs* args, hipStream_t stream) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
        if (n_cu <= 0) n_cu = 256;
    }
    bgx::MovegenArgs a = *args;
    if (a.n_jobs <= 0 && !a.n_jobs_dev) return hipSuccess;
    hipError_t e = hipMemsetAsync(a.ovf_count, 0, sizeof(unsigned), stream);
    if (e != hipSuccess) return e;
    // persistent grid: at most 2 resident 4-wave blocks per CU (80 KB LDS each), x4 rounds
    int blocks = n_cu * 8;
    if (!a.n_jobs_dev) {
        const int need = (a.n_jobs + 3) / 4;
        if (need < blocks) blocks = need;
    }
    hipLaunchKernelGGL(bgx::movegen_lds_kernel, dim3(blocks), dim3(256), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bgx::movegen_global_kernel, dim3(a.ws_waves), dim3(64), 0, stream, a);
    return hipGetLastError();
}
