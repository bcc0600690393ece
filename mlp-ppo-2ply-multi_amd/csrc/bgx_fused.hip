// bgx_fused.hip — the 1-ply self-play step fused into one persistent launch.
//
// One workgroup owns 16 or 32 game lanes (FL) and runs n_steps env steps of
// each, with no kernel boundary between the steps. 8 wavefronts per workgroup
// (256 registers each):
//   1. movegen: the waves take the workgroup's (board, player, dice) jobs
//      from an LDS queue (doubles first) and expand each in their own 4 KB LDS slice (tier 1, bgx_movegen.h) and
//      writes the afterstates to the lane's candidate slots; a job that
//      outgrows the slice is redone after the barrier (tier 2: a doubles job
//      outside bear-off by the whole workgroup's path expansion, else a 32 KB
//      slice in wave 0; tier 3: the workgroup's global workspace), as
//      movegen_block_kernel does;
//   2. the LDS that held the slices takes the split-fp16 W fragments, and the
//      workgroup's rows (the lanes' obs rows + candidates, ~340 per step) are
//      staged behind them;
//   3. value MLP in 32-board tile items spread over the waves, all four
//      32-hidden m-tiles of a tile in one wave (mlp_tile4; the canonical
//      epilogue order, so V has the same bits as the phased engine's) — V
//      lands in LDS;
//   4. each wave samples its lanes' actions from softmax(V/T) and runs the env
//      step (lane_advance: apply, rewards, record, reset) on the lane state,
//      which stays in LDS for the whole launch.
// Replaces, per lane and step, Worker.play_episode's inner loop
// (src/multi/worker.py:101-162) over BackgammonEnv.step / update_legal_moves
// (src/environments/backgammon_env.py:130-308) and the policy forward
// (src/agents/policy_network.py:53-70), exactly as the phased engine
// (bgx_abi.cpp enqueue_steps: movegen, mlp, select_step) does; the lanes of a
// workgroup wait only for each other at the barriers, never for the other
// 4,000 lanes, and there is no per-step launch.
#include "bgx_engine.h"
#include "bgx_mlp.h"
#include "bgx_movegen.h"

namespace bgx {

// FL = game lanes per workgroup and NW = waves per workgroup: 16 lanes on 8
// waves (2 per SIMD, 256 registers) when fewer lanes than 32 x CUs, else 32
// lanes on 12 waves (3 per SIMD, 168 registers): the tier-1 queue then holds
// 32 jobs, so the long doubles jobs of a step are spread over more short ones,
// and a third wave per SIMD hides more of each job's latency.
// LDS: [scratch | W fragments (resident for the launch) | tail | lane values]
//  scratch = NW tier-1 slices (the pool kernel's layout, bgx_movegen.hip: a
//  64-word parent map + a region holding the table-mode or the table-free
//  lists; 4 KB at 8 waves, 3.5 KB at 12) during movegen, the 32 KB tier-2
//  slice, then the MLP partials + staged rows
template <int FL> struct FusedTail {
    uint4 lut[256];                 // feature LUT (bgx_mlp.h lut_entry)
    float w2s[128];                 // value-head weights
    int cnt[FL];                    // lane's full candidate count this step (-1: redo in tier 2)
    int next[2];                    // tier-1 job counters, alternating by step parity
    int bdone;                      // last-round lanes stepped so far (this group; see OVL)
    int go[2];                      // step s runs iff go[s & 1] (the balanced launch's tickets)
    int qnext;                      // the merged MLP + choice phase's item counter
    unsigned tdone[64];             // MLP tile t of this step is written iff tdone[t] == the step's tag
    int pre[FL + 1];                // MLP row prefix over the lanes
    uint32_t job[FL][8];            // the lanes' jobs: packed board words 0..6, player | d0 << 8 | d1 << 16
    LaneState st[FL];               // the lanes' state for the whole launch (written back at the end)
};
template <int FL> struct FCfg {
    static constexpr int NW = FL == 32 ? 12 : 8;
    static constexpr int WPE = NW / 4;                   // waves per SIMD
    // (a 128-slot table with 288-entry frontiers at 12 waves: more tier-2 jobs, not faster)
    static constexpr int P1_S = 256, P1_F = NW > 8 ? 160 : 224, P1_PF = NW > 8 ? 416 : 480;
    static constexpr int SL1 = 64 * 4 + 2 * P1_PF * 4;
    static_assert(P1_S * 8 + 2 * P1_F * 4 <= 2 * P1_PF * 4, "table layout fits the region");
    static constexpr int F_SCR = NW * SL1 > Slice<S_T2>::bytes ? NW * SL1 : Slice<S_T2>::bytes;
    static constexpr int F_W = F_SCR;
    // tier 2 of a doubles path job: the whole workgroup over the scratch
    static constexpr int CP_F = 128 * NW;
    static_assert(sizeof(CoopPathLds<NW, CP_F>) <= F_SCR, "path expansion fits the scratch");
    static constexpr int F_TAIL = F_W + NFRAG * 16;
    static constexpr int FT = F_SCR / (32 * 32);   // MLP tiles per batch: staged rows (32 B per board)
    static_assert(FT <= 64, "a tile flag per staged tile (FusedTail::tdone)");
    // V(s), V(candidates 0..XS-2) of each lane kept in LDS (the rest: vbuf): as many as fit (<= 96)
    static constexpr int XS_FIT = (160 * 1024 - F_TAIL - (int)sizeof(FusedTail<FL>)) / (FL * 4);
    static constexpr int XS = XS_FIT < 96 ? XS_FIT : 96;
    static constexpr int LDS = F_TAIL + (int)sizeof(FusedTail<FL>) + FL * XS * 4;
    static_assert(XS >= 24 && LDS <= 160 * 1024, "fits the CU's LDS");
};

template <bool PROF, int FL>
__global__ __launch_bounds__(64 * FCfg<FL>::NW, FCfg<FL>::WPE) void fused_step_kernel(FusedArgs f) {
    using C = FCfg<FL>;
    constexpr int NW = C::NW, SL1 = C::SL1, F_W = C::F_W, F_TAIL = C::F_TAIL, FT = C::FT, XS = C::XS;
    constexpr int P1_S = C::P1_S, P1_F = C::P1_F, P1_PF = C::P1_PF;
    constexpr int CP_F = C::CP_F;
    // the cooperative tier 2 at 12 waves only (at 8 waves, 256 registers, its
    // registers spill in the step loop: 0 -> 19)
    constexpr bool COOP2 = NW > 8;
    constexpr int NT = 64 * NW;          // threads
    constexpr int PR = (FL + 2 * NW - 1) / (2 * NW);   // rounds of the choice phase (two lanes per wave each)
    // OVL: the choice phase's last round is partial (32 lanes on 12 waves: 24 +
    // 8); it runs without a barrier behind it, so the waves it leaves idle start
    // the next step's tier-1 jobs of the NA lanes already stepped, and a job of
    // a last-round lane waits (LDS counter T.bdone) until those lanes are stepped
    constexpr bool OVL = PR >= 2 && FL < 2 * NW * PR;
    constexpr int NA = OVL ? 2 * NW * (PR - 1) : FL;
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    uint8_t* lds = (uint8_t*)smem;
    FusedTail<FL>& T = *(FusedTail<FL>*)(lds + F_TAIL);
    float* xs = (float*)(lds + F_TAIL + sizeof(FusedTail<FL>));   // [FL][XS] lane values
    const EngineDev& e = f.e;
    const int t = (int)threadIdx.x, w = t >> 6, l = lane_id();
    for (int i = t; i < 256; i += NT) T.lut[i] = lut_entry((uint32_t)i, f.feat_scale);
    for (int i = t; i < 128; i += NT) T.w2s[i] = f.rowc[i];
    for (int i = t; i < 64; i += NT) T.tdone[i] = 0u;
    unsigned qtag = 0u;   // this workgroup's step counter (tags tdone; never 0 on a live step)
    uint4* wl = (uint4*)(lds + F_W);     // split-fp16 W fragments, loaded once
    for (int k = t; k < NFRAG; k += NT) wl[k] = f.wfrag[k];
    const uint4* wf = wl;

    MovegenArgs a{};
    a.out_mode = OUT_PACKED_SLOT;
    a.cap = f.cap;
    a.out_packed = f.cand;
    a.out_count = const_cast<int32_t*>(e.cand_cnt);
    a.ws_global = f.ws_global;
    a.ws_slots = f.ws_slots;
    a.ws_words_per_wave = f.ws_words_per_block;
    a.heavy_t = 0x7FFFFFFF;
    a.force_tier = f.force_tier;
    a.err_flags = e.err_flags;

    unsigned long long n_rows = 0, n_fb = 0, n_steps = 0;
    const unsigned long long wg_begin = PROF ? wall_clock64() : 0ull;   // this launch's span (f.prof)
    // development timers (f.prof): phase sums on thread 0, per-wave sums on lane 0
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tj = 0, tc = 0, tw[4] = {0, 0, 0, 0}, t2c = 0, t3n = 0;
    unsigned long long tjd[4] = {0, 0, 0, 0};   // tier-1 job clocks / counts: doubles, non-doubles
    unsigned long long twb = 0;                 // tier-1 clocks spent waiting for the last-round lanes
    unsigned long long tpre = 0;                // tier-1 clocks from a job's queue pop to its expansion
    unsigned long long tpa = 0, tpm = 0;        // ... of which: queue pop + lane lookup, job words + root analysis
    unsigned long long tcs[3] = {0, 0, 0};      // choice: state + Philox refill, pick, env step (lane_advance)
    constexpr bool prof = PROF;
    auto tick = [&](int k) {
        if (prof && t == 0) {
            const unsigned long long c = wall_clock64();
            ph[k] += c - tc;
            tc = c;
        }
    };
    uint4* rs = (uint4*)lds;                           // [FT * 32][2] staged rows (scratch)
    const int groups = (e.L + FL - 1) / FL;
    for (int g = (int)blockIdx.x; g < groups; g += (int)gridDim.x) {
        const int nlive = e.L - g * FL < FL ? e.L - g * FL : FL;
        for (int v = t; v < nlive; v += NT) lane_load(e, g * FL + v, T.st[v]);
        if (t == 0) {
            T.next[0] = T.next[1] = NW;
            T.bdone = 0;
        }
        const int na = nlive < NA ? nlive : NA, nbl = nlive - na;   // lanes stepped before / in the last round
        // step s runs iff ticket(s): lockstep, s < n_steps; balanced, s < n_cap and
        // the launch's lane-step total before this workgroup-step is below the
        // budget (thread 0 takes step s + 1's ticket late in step s, before the
        // MLP phase's last barrier, which publishes it: a workgroup commits to a
        // further step as late as the choice phase allows, so the launch's tail
        // after the budget runs out is about one step)
        auto ticket = [&](int s) -> int {
            if (f.budget <= 0) return s < f.n_steps;
            if (s >= f.n_cap) return 0;
            const unsigned long long old = atomicAdd(f.budget_ctr, (unsigned long long)nlive);
            return old < (unsigned long long)f.budget;
        };
        if (t == 0) T.go[0] = ticket(0);
        __syncthreads();
        const int n_iter = f.budget > 0 ? f.n_cap : f.n_steps;
        for (int step = 0; step < n_iter && T.go[step & 1]; ++step) {
            n_steps += (unsigned long long)nlive;
            // ---- 1. tier-1 movegen of the wave's lanes in its slice
            if (prof && t == 0) tc = wall_clock64();
            {
                const unsigned long long j0 = prof ? wall_clock64() : 0ull;
                uint32_t* sl = (uint32_t*)(lds + (size_t)w * SL1);
                Mem M;
                M.map = sl;
                M.tab = (unsigned long long*)(sl + 64);
                M.S = P1_S;
                M.F = P1_F;
                M.fa = sl + 64 + 2 * P1_S;
                M.fb = M.fa + P1_F;
                M.pa = sl + 64;
                M.pb = M.pa + P1_PF;
                M.PF = P1_PF;
                M.map[l] = 0u;
                wave_sync();
                // the workgroup's jobs in a queue, doubles (the long jobs) first; each
                // wave takes the next one from an LDS counter until none is left.
                // The loop holds no workgroup barrier (the tiers that need one run
                // after it), its index is wave-uniform (lane 0's atomic, read back
                // with readfirstlane) and only grows, so every wave leaves it.
                // (OVL: queue = the NA lanes stepped before the last round, doubles
                // first, then the last-round lanes, doubles first, read once they are stepped)
                const bool dbl = l < na && T.st[l].d0 == T.st[l].d1;
                const uint32_t dmask = (uint32_t)ballot(dbl), omask = (uint32_t)ballot(l < na && !dbl);
                const int nd = __popc(dmask);
                uint32_t dmb = 0u, omb = 0u;
                int ndb = -1;
                int* next = &T.next[step & 1];
                // wave w starts with job w; the counter (preset to NW) hands out the
                // rest; at most FL iterations, whatever the counter returns
                int k = w;
                for (int it = 0; it < FL && k < nlive; ++it) {
                    const unsigned long long it0 = prof ? wall_clock64() : 0ull;
                    int kn = 0;
                    if (l == 0) kn = atomicAdd(next, 1);
                    kn = uniform(kn);
                    int v;
                    if (!OVL || k < na) {
                        v = k < nd ? select_bit(dmask, k) : select_bit(omask, k - nd);
                    } else {
                        if (ndb < 0) {
                            // the last-round lanes of the previous step: every one
                            // is stepped by a wave that has no barrier ahead of it
                            const int target = step * nbl;
                            const unsigned long long b0 = prof ? wall_clock64() : 0ull;
                            // bounded: the lanes' waves have no barrier ahead, so
                            // the wait ends; if a change ever breaks that, the bound turns the hang
                            // into BGX_E_STATE at bgx_sync instead of a stuck GPU
                            for (unsigned spin = 0;
                                 __hip_atomic_load(&T.bdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target;
                                 ++spin) {
                                if (spin >= (1u << 24)) {
                                    if (l == 0) atomicOr(e.err_flags, BGX_ERRF_WAIT_BOUND);
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(1);
                            }
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                            if (prof) twb += wall_clock64() - b0;
                            const bool inb = l >= na && l < nlive;
                            const bool db = inb && T.st[l].d0 == T.st[l].d1;
                            dmb = (uint32_t)ballot(db);
                            omb = (uint32_t)ballot(inb && !db);
                            ndb = __popc(dmb);
                        }
                        const int kb = k - na;
                        v = kb < ndb ? select_bit(dmb, kb) : select_bit(omb, kb - ndb);
                    }
                    const unsigned long long ia = prof ? wall_clock64() : 0ull;
                    if (prof) tpa += ia - it0;
                    const LaneState& st = T.st[v];
                    if (l < 8)
                        T.job[v][l] = l < 7 ? st.w[l] : (uint32_t)st.p | ((uint32_t)st.d0 << 8) | ((uint32_t)st.d1 << 16);
                    STAMP_BEGIN;
                    const JobIn in =
                        make_job(st.w[0], st.w[1], st.w[2], st.w[3], st.w[4], st.w[5], st.w[6], st.p, st.d0, st.d1);
                    STAMP(in.d0 == in.d1 ? 5 : 0);
                    if (prof) {
                        // make the root analysis finish before the clock (its first use)
                        __builtin_amdgcn_s_waitcnt(0);
                        tpm += wall_clock64() - ia;
                    }
                    uint32_t* fin = nullptr;
                    const unsigned long long q0 = prof ? wall_clock64() : 0ull;
                    if (prof) tpre += q0 - it0;
                    const int nf = f.force_tier >= 2 ? -1 : job_records<false>(in, M, fin, 0x7FFFFFFF);
                    STAMP(in.d0 == in.d1 ? 12 : 13);
                    if (nf >= 0) emit_records<false>(a, g * FL + v, in, fin, nf, 0);
                    STAMP(in.d0 == in.d1 ? 10 : 3);
#ifdef BGX_STAMP
                    if (nf >= 0 && l == 0) atomicAdd(&bgx_stamp_acc[(blockIdx.x & 255) * 32 + (in.d0 == in.d1 ? 15 : 14)], (unsigned long long)nf);
#endif
                    wave_sync();
                    if (l == 0) T.cnt[v] = nf;
                    if (prof) {
                        const int kd = in.d0 == in.d1 ? 0 : 2;
                        tjd[kd] += wall_clock64() - q0;
                        tjd[kd + 1] += 1;
                    }
                    k = kn;
                }
                if (prof) tj += wall_clock64() - j0;
            }
            __syncthreads();
            if (t == 0) T.next[(step + 1) & 1] = NW;   // the next step's counter (last used two steps ago)
            tick(0);
            // ---- 1b. jobs that outgrew their slice: the workgroup, one at a time (rare)
            const int cnt_l = l < nlive ? T.cnt[l] : 0;   // lane q < 16 holds lane q's count
            uint32_t ovf = (uint32_t)ballot(l < FL && cnt_l < 0);
            while (ovf) {
                const int v = __ffs(ovf) - 1;
                ovf &= ovf - 1u;
                ++n_fb;
                const unsigned long long c2 = prof ? wall_clock64() : 0ull;
                const int j = g * FL + v;
                const uint32_t* q = T.job[v];
                const JobIn in = make_job(q[0], q[1], q[2], q[3], q[4], q[5], q[6], (int)(q[7] & 255u),
                                          (int)((q[7] >> 8) & 255u), (int)(q[7] >> 16));
                FlatCursor fc;
                auto run_global = [&]() -> int {
                    uint32_t* base = f.ws_global + (size_t)blockIdx.x * f.ws_words_per_block;
                    Mem G;
                    const int S = f.ws_slots;
                    G.tab = (unsigned long long*)base;
                    G.fa = base + 2 * S;
                    G.fb = base + 3 * S;
                    G.map = base + 4 * S;
                    G.S = S;
                    G.F = S;
                    st32<true>(G.map + l, 0u);
                    sync<true>();
                    if (prof) ++t3n;
                    const int r = run_job<true>(a, j, in, G, fc);
                    if (r < 0 && l == 0) atomicOr(e.err_flags, BGX_ERRF_FALLBACK_OVERFLOW);
                    return r < 0 ? 0 : r;
                };
                // tier 2 of a doubles job outside bear-off / the bar: the path
                // expansion by every wave over the scratch, then each wave emits
                // every NW-th chunk of the records
                int r2 = -1;
                if (COOP2 && in.d0 == in.d1 && doubles_by_path(in.R) && f.force_tier < 3) {
                    auto& C = *(CoopPathLds<NW, CP_F>*)lds;
                    uint32_t* fin = nullptr;
                    r2 = coop_doubles_path<NW, CP_F>(in, C, fin);
                    if (r2 >= 0) {
                        emit_records<false>(a, j, in, fin, r2, 0, 64 * w, 64 * NW);
                        if (t == 0) {
                            T.cnt[v] = r2;
                            a.out_count[j] = r2;
                        }
                    }
                    __syncthreads();
                }
                if (r2 < 0 && w == 0) {   // tier 2: a 32 KB slice in wave 0, then tier 3
                    const Mem M2 = lds_mem<S_T2>(smem);
                    int r = f.force_tier >= 3 ? -1 : run_job<false>(a, j, in, M2, fc);
                    if (r < 0) r = run_global();
                    if (l == 0) T.cnt[v] = r;
                }
                __syncthreads();
                if (prof) t2c += wall_clock64() - c2;
            }
            // ---- 2. row prefix (lanes that pass evaluate nothing), every wave
            // computes it (identical values; no barrier needed before its use)
            {
                const int c = l < nlive ? T.cnt[l] : 0;
                const int rows = l < FL && c > 0 ? 1 + (c < f.cap ? c : f.cap) : 0;
                const int incl = wave_incl_scan(rows);
                if (l <= FL) T.pre[l] = incl - rows;
                wave_sync();
            }
            tick(1);
            const int nr = T.pre[FL];
            n_rows += (unsigned long long)nr;
            // row r of the workgroup -> its lane: the last v with pre[v] <= r
            // (binary search; lanes without rows have pre[v] == pre[v + 1])
            auto lane_of = [&](int r) -> int {
                int v = 0;
#pragma unroll
                for (int step = FL / 2; step >= 1; step >>= 1)
                    if (T.pre[v + step] <= r) v += step;
                return v;
            };
            auto stage = [&](int tb, int nt) {   // rows of tiles tb.. into LDS, all loads in flight together
                for (int c = t; c < nt * 32; c += NT) {
                    const int r = tb * 32 + c;
                    uint4 bx = make_uint4(0, 0, 0, 0), by = make_uint4(0, 0, 0, 0);
                    if (r < nr) {
                        const int v = lane_of(r), k = r - T.pre[v];
                        const int li = g * FL + v;
                        const uint32_t* src =
                            k == 0 ? e.rows + (size_t)li * 8 : f.cand + ((size_t)li * f.cap + (k - 1)) * 8;
                        bx = ((const uint4*)src)[0];
                        by = ((const uint4*)src)[1];
                    }
                    rs[2 * c] = bx;
                    rs[2 * c + 1] = by;
                }
            };
            // ---- 5 (body). action choice + env step of lane v (the chosen
            // afterstate is still staged in LDS when the step fit one MLP batch
            // and this is not the OVL round); two of a wave's lanes side by side,
            // one per half-wave
            auto choose = [&](int v, bool last) {
                const bool lead = (l & 31) == 0;
                if (v < nlive) {
                const int i = g * FL + v;
                const unsigned long long s1 = prof ? wall_clock64() : 0ull;
                LaneState sr = T.st[v];
                const int n_full = T.cnt[v];
                const int n = n_full < e.max_legal ? n_full : e.max_legal;
                HalfRng rng;
                rng.key = lane_key(e.seed, (uint32_t)(e.lane_base + i));
                rng.ctr = sr.ctr;
                rng.dt = lane_dice(e, i);
                rng.refill();
                unsigned long long c0 = 0;
                if (prof) {
                    __builtin_amdgcn_s_waitcnt(0);
                    c0 = wall_clock64();
                    tcs[0] += c0 - s1;
                }
                if (n <= 0) {
                    lane_advance(e, i, sr, rng, -1, sr.w, 0.0f, 0.0f, 0, lead);
                } else {
                    const float* xv = xs + v * XS;   // V(s), then V(candidate k) at 1 + k
                    const float* vv = f.vbuf + (size_t)i * (f.cap + 1);
                    const float Tm = e.temperature;
                    const float u = unit_from(rng.at(0).x);   // lane_uniform: Philox at the lane's counter
                    const int pick =
                        n + 1 <= XS
                            ? pick_action_half([&](int k) { return xv[1 + k] / Tm; }, n, e.greedy != 0, u)
                            : pick_action_half([&](int k) { return (1 + k < XS ? xv[1 + k] : vv[1 + k]) / Tm; }, n,
                                               e.greedy != 0, u);
                    if (prof) {
                        const unsigned long long c1 = wall_clock64();
                        tw[2] += c1 - s1;
                        tcs[1] += c1 - c0;
                        c0 = c1;
                    }
                    uint32_t nb[8];
                    const int r = T.pre[v] + 1 + pick;
                    if (nr <= FT * 32 && !last) {
                        const uint4 bx = rs[2 * r], by = rs[2 * r + 1];
                        nb[0] = bx.x; nb[1] = bx.y; nb[2] = bx.z; nb[3] = bx.w;
                        nb[4] = by.x; nb[5] = by.y; nb[6] = by.z; nb[7] = by.w;
                    } else {
                        load_packed(f.cand + ((size_t)i * f.cap + pick) * 8, nb);
                    }
                    const float va = 1 + pick < XS ? xv[1 + pick] : vv[1 + pick];
                    lane_advance(e, i, sr, rng, pick, nb, xv[0], va, n_full, lead);
                    if (prof) {
                        __builtin_amdgcn_s_waitcnt(0);
                        tcs[2] += wall_clock64() - c0;
                    }
                }
                wave_sync();
                if (lead) T.st[v] = sr;
                if (last && lead) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    atomicAdd(&T.bdone, 1);
                }
                if (prof) tw[3] += wall_clock64() - s1;
                }
            };
            // one MLP tile (32 rows) of batch tb: V into the lanes' values
            auto mlp_one = [&](int tb, int it) {
                const int c0 = it * 32 + (l & 31);
                const uint4 bx = rs[2 * c0], by = rs[2 * c0 + 1];
                const float v = mlp_tile4(wf, T.lut, T.w2s, f.feat_scale, bx, by, tile_kmask(bx, by));
                const int r = (tb + it) * 32 + l;
                if (l < 32 && r < nr) {
                    const float val = v + f.b2;
                    const int vl = lane_of(r), k = r - T.pre[vl];
                    if (k < XS) xs[vl * XS + k] = val;
                    else f.vbuf[(size_t)(g * FL + vl) * (f.cap + 1) + k] = val;
                }
            };
            // ---- 3. the first batch's rows into the scratch
            const int n_tiles = (nr + 31) >> 5;
            // one batch (the usual case): the MLP tiles and the choice phase's
            // first round are one item queue (below)
#ifdef BGX_NO_MERGE
            const bool merged = false;   // A/B builds: barrier-separated MLP and choice phases
#else
            const bool merged = n_tiles <= FT;
#endif
            stage(0, n_tiles < FT ? n_tiles : FT);
            if (t == 0) T.qnext = NW;
            if (n_tiles == 0 && t == 0) T.go[(step + 1) & 1] = ticket(step + 1);   // no MLP batch this step
            ++qtag;
            __syncthreads();
            tick(2);
            const unsigned long long m0 = prof ? wall_clock64() : 0ull;
            if (merged) {
                // ---- 4 + 5a. value MLP and the first choice round as one queue:
                // items 0 .. n_tiles - 1 are the MLP tiles (one 32-board tile per
                // item, all four m-tiles in the wave: mlp_tile4), then one item per
                // pair of first-round lanes. A wave takes item w, then the next from
                // an LDS counter; a choice item waits (LDS flags, bounded) for the
                // tiles holding its lanes' rows. Every tile item is handed out before
                // any choice item and a tile item waits on nothing, so the waits end.
                // The MFMA-bound tiles and the latency-bound choice chains then share
                // the SIMDs instead of running in two barrier-separated phases.
                const int nc0 = (nlive + 1) / 2 < NW ? (nlive + 1) / 2 : NW;   // first-round lane pairs
                int it = w;
                while (it < n_tiles + nc0) {
                    if (it < n_tiles) {
                        const unsigned long long i0 = prof ? wall_clock64() : 0ull;
                        mlp_one(0, it);
                        // the tile's values (LDS and, past XS, vbuf) before its flag
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (l == 0) __hip_atomic_store(&T.tdone[it], qtag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (prof) tw[1] += wall_clock64() - i0;
                    } else {
                        const int p = it - n_tiles;
                        const int va = 2 * p, vb = 2 * p + 2 < nlive ? 2 * p + 2 : nlive;
                        const int r0 = T.pre[va], r1 = T.pre[vb];   // the pair's rows [r0, r1)
                        if (r1 > r0) {
                            for (int tt = r0 >> 5; tt <= (r1 - 1) >> 5; ++tt) {
                                // bounded like every in-kernel wait
                                for (unsigned spin = 0;
                                     __hip_atomic_load(&T.tdone[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != qtag;
                                     ++spin) {
                                    if (spin >= (1u << 24)) {
                                        if (l == 0) atomicOr(e.err_flags, BGX_ERRF_WAIT_BOUND);
                                        break;
                                    }
                                    __builtin_amdgcn_s_sleep(1);
                                }
                            }
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                        }
                        choose(2 * p + (l >> 5), false);
                    }
                    int kn = 0;
                    if (l == 0) kn = atomicAdd(&T.qnext, 1);
                    it = uniform(kn);
                }
                // (no barrier here: the OVL round starts with one, and without OVL
                // the step ends with one)
                if (n_tiles > 0 && t == 0) T.go[(step + 1) & 1] = ticket(step + 1);
            } else {
                // ---- 4. value MLP over FT-tile batches (many rows this step)
                for (int tb = 0; tb < n_tiles; tb += FT) {
                    const int nt = n_tiles - tb < FT ? n_tiles - tb : FT;
                    const unsigned long long i0 = prof ? wall_clock64() : 0ull;
                    for (int it = w; it < nt; it += NW) mlp_one(tb, it);
                    if (prof) tw[1] += wall_clock64() - i0;   // the wave's MLP items (no barrier)
                    if (tb + FT >= n_tiles && t == 0) T.go[(step + 1) & 1] = ticket(step + 1);   // the last batch
                    __syncthreads();
                    if (tb + FT < n_tiles) {
                        stage(tb + FT, n_tiles - tb - FT < FT ? n_tiles - tb - FT : FT);
                        __syncthreads();
                    }
                }
            }
            if (prof) tw[0] += wall_clock64() - m0;
            tick(3);
            // ---- 5. the remaining choice rounds (all of them after a multi-batch MLP)
#pragma unroll 1
            for (int pr = merged ? 1 : 0; pr < PR; ++pr) {
                const bool last = OVL && pr == PR - 1;
                if (last) __syncthreads();   // the staged rows are the next step's slices from here on
                choose(2 * (pr * NW + w) + (l >> 5), last);
            }
            // the next step's ticket (written before this step's first barrier):
            // the OVL round's lanes are finished by a barrier before the group ends
            if (!OVL || !T.go[(step + 1) & 1]) __syncthreads();
            tick(4);
            if (prof && t == 0) ph[5] += 1;
        }
        for (int v = t; v < nlive; v += NT) lane_store(e, g * FL + v, T.st[v]);
        __syncthreads();
    }
    if (prof) {
        unsigned long long* P = f.prof + (size_t)blockIdx.x * 32;
        if (t == 0) {
            // the last launch's begin / end clocks, rows and tier-2 jobs of this
            // workgroup (overwritten per launch: the spread of the workgroups'
            // durations is what a short launch waits for)
            P[24] = wg_begin;
            P[25] = wall_clock64();
            P[26] = n_rows;
            P[27] = n_fb;
            P[28] = n_steps;
            for (int k = 0; k < 6; ++k) atomicAdd(P + k, ph[k]);
            atomicAdd(P + 11, t2c);
            atomicAdd(P + 12, n_fb);
            atomicAdd(P + 13, t3n);
            atomicAdd(P + 18, (unsigned long long)NW * ph[5]);   // wave-steps
        }
        if (l == 0) {
            atomicAdd(P + 6, tj);
            for (int k = 0; k < 4; ++k) atomicAdd(P + 7 + k, tw[k]);
            for (int k = 0; k < 4; ++k) atomicAdd(P + 14 + k, tjd[k]);
            atomicAdd(P + 19, twb);
            atomicAdd(P + 20, tpre);
            atomicAdd(P + 21, tpa);
            atomicAdd(P + 22, tpm);
            for (int k = 0; k < 3; ++k) atomicAdd(P + 29 + k, tcs[k]);
        }
    }
    if (t == 0) {
        atomicAdd(e.stats + 0, n_steps);
        atomicAdd(e.stats + 3, n_rows);
        atomicAdd(e.stats + 4, n_steps);
        atomicAdd(e.stats + 5, n_fb);
        if (f.budget > 0) {
            // the last workgroup to finish zeroes the lane-step counter for the
            // next launch (stream order: no memset launch in between)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (atomicAdd(f.budget_ctr + 1, 1ull) == (unsigned long long)gridDim.x - 1ull) {
                __hip_atomic_store(f.budget_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(f.budget_ctr + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

}  // namespace bgx

#ifdef BGX_STAMP
// diagnostic builds: the section sums over all CU slots (then zeroed)
extern "C" int bgx_diag_stamps(unsigned long long* out32) {
    static unsigned long long h[256 * 32];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(bgx::bgx_stamp_acc), sizeof(h)) != hipSuccess) return -1;
    for (int k = 0; k < 32; ++k) {
        out32[k] = 0;
        for (int b = 0; b < 256; ++b) out32[k] += h[b * 32 + k];
    }
    static unsigned long long z[256 * 32];
    return hipMemcpyToSymbol(HIP_SYMBOL(bgx::bgx_stamp_acc), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" hipError_t bgx_launch_fused(const bgx::FusedArgs* args, hipStream_t stream) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
        const void* k16[] = {(const void*)bgx::fused_step_kernel<false, 16>, (const void*)bgx::fused_step_kernel<true, 16>};
        const void* k32[] = {(const void*)bgx::fused_step_kernel<false, 32>, (const void*)bgx::fused_step_kernel<true, 32>};
        for (const void* k : k16)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bgx::FCfg<16>::LDS) != hipSuccess)
                return hipErrorInvalidValue;
        for (const void* k : k32)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bgx::FCfg<32>::LDS) != hipSuccess)
                return hipErrorInvalidValue;
    }
    if (args->n_steps <= 0 || args->e.L <= 0) return hipSuccess;
    if (args->cap < 1 || args->cap > 2048) return hipErrorInvalidValue;
    // persistent: one workgroup per CU (LDS, registers) and one tier-3 slice each;
    // 32 lanes per workgroup when that still gives every CU a workgroup
    const int L = args->e.L;
    const int fl = args->lanes_per_wg == 16 || args->lanes_per_wg == 32 ? args->lanes_per_wg
                   : ((L + 31) / 32 >= n_cu ? 32 : 16);
    const int groups = (L + fl - 1) / fl;
    int blocks = groups < n_cu ? groups : n_cu;
    if (blocks > args->ws_blocks) blocks = args->ws_blocks;
    const dim3 g(blocks), b(64 * (fl == 32 ? bgx::FCfg<32>::NW : bgx::FCfg<16>::NW));
    bgx::FusedArgs a = *args;
    // balanced only when every workgroup owns one lane group (a workgroup that
    // walks several groups would spend the budget on its first ones)
    if (a.budget > 0 && (groups > blocks || !a.budget_ctr || a.n_cap < a.n_steps)) a.budget = 0;
    if (fl == 32) {
        if (a.prof)
            hipLaunchKernelGGL((bgx::fused_step_kernel<true, 32>), g, b, bgx::FCfg<32>::LDS, stream, a);
        else
            hipLaunchKernelGGL((bgx::fused_step_kernel<false, 32>), g, b, bgx::FCfg<32>::LDS, stream, a);
    } else {
        if (a.prof)
            hipLaunchKernelGGL((bgx::fused_step_kernel<true, 16>), g, b, bgx::FCfg<16>::LDS, stream, a);
        else
            hipLaunchKernelGGL((bgx::fused_step_kernel<false, 16>), g, b, bgx::FCfg<16>::LDS, stream, a);
    }
    return hipGetLastError();
}
