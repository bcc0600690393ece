// bgx_fused.hip — the 1-ply self-play step fused into one persistent launch.
//
// One workgroup owns 16 or 32 game lanes (FL) and runs n_steps env steps of
// each, with no kernel boundary between the steps. Per step s:
//   1b. jobs whose tier-1 expansion outgrew the wave's slice are redone by the
//      workgroup (tier 2: a doubles job outside bear-off by the whole
//      workgroup's path expansion, else a 32 KB slice in wave 0; tier 3: the
//      workgroup's global workspace), as movegen_block_kernel does;
//   2. the lanes' row prefix (obs row + candidates of each lane);
//   3. one LDS item queue, taken by the waves in order: the step's MLP tiles
//      (32 boards each, all four 32-hidden m-tiles in one wave: mlp_tile4, the
//      canonical epilogue order, so V has the phased engine's bits; V lands in
//      LDS), then its choice items (two lanes per wave, one per half-wave:
//      softmax(V/T) sample and the env step lane_advance -- apply, rewards,
//      record, reset -- on the LDS-resident lane state), then step s + 1's
//      tier-1 movegen jobs (one lane each, in the wave's own LDS slice,
//      bgx_movegen.h, afterstates into the lane's candidate slots). A choice
//      waits for the tiles holding its lanes' rows, a job for its lane's
//      choice (LDS flags); the MFMA-bound tiles, the latency-bound choices and
//      the issue-bound movegen jobs share the SIMDs.
// Replaces, per lane and step, Worker.play_episode's inner loop
// (src/multi/worker.py:101-162) over BackgammonEnv.step / update_legal_moves
// (src/environments/backgammon_env.py:130-308) and the policy forward
// (src/agents/policy_network.py:53-70), exactly as the phased engine
// (bgx_abi.cpp enqueue_steps: movegen, mlp, select_step) does; the lanes of a
// workgroup wait only for each other, never for the other 8,000 lanes, and
// there is no per-step launch.
#include "bgx_engine.h"
#include "bgx_mlp.h"
#include "bgx_movegen.h"

#ifndef BGX_FUSED_NW32
#define BGX_FUSED_NW32 12   // waves per 32-lane workgroup (12: 3 per SIMD at 168 registers; 8: 2 per SIMD at 256; A/B)
#endif
#ifndef BGX_FUSED_NW16
#define BGX_FUSED_NW16 12   // waves per 16-lane workgroup (fewer lanes than 32 x CUs; 8 measured 6 % slower; A/B)
#endif
#ifndef BGX_HALF_TICKETS
#define BGX_HALF_TICKETS 0   // 1: half-lane tickets in a balanced launch's last round (measured slower: DESIGN.md section 9; A/B)
#endif
#ifndef BGX_FUSED_LEAF
#define BGX_FUSED_LEAF 0   // A/B builds: 1 = tier-1 path doubles stream their leaves (run_job<LEAF>)
#endif

namespace bgx {

constexpr int PROF_STRIDE = 128;   // u64 words per workgroup slot of the development report (f.prof)

// FL = game lanes per workgroup and NW = waves per workgroup: 16 lanes when
// fewer lanes than 32 x CUs, else 32 lanes (a step's queue then holds 32 jobs,
// so the long doubles jobs are spread over more short ones); both on 12 waves
// (3 per SIMD, 168 registers): the third wave per SIMD hides more of each
// item's latency than the spills it costs (32 lanes on 8 waves 270 -> 226 M,
// 16 lanes on 8 waves at 4,096 lanes 216 -> 203 M).
// LDS: [scratch | W fragments (resident for the launch) | tail | lane values]
//  scratch = NW tier-1 slices (the pool kernel's layout, bgx_movegen.hip: a
//  64-word parent map + a region holding the table-mode or the table-free
//  lists; 4 KB at 8 waves, 3.5 KB at 12), or the workgroup's tier-2 space
template <int FL> struct FusedTail {
    uint4 lut[256];                 // feature LUT (bgx_mlp.h lut_entry)
    float w2s[128];                 // value-head weights
    int cnt[FL];                    // lane's full candidate count this step (-1: redo in tier 2)
    int go[2];                      // step s runs iff go[s & 1] (the balanced launch's tickets)
    int qn[2];                      // the step queue's item counters (by pass parity)
    unsigned tdone[64];             // MLP tile t of this step is written iff tdone[t] == the step's tag
    unsigned chosen[FL];            // lane v of this step is stepped iff chosen[v] == the step's tag
    unsigned claim[FL];             // lane v's next tier-1 job is taken iff claim[v] == the step's tag
    int pre[FL + 1];                // MLP row prefix over the lanes
    uint32_t job[FL][8];            // the lanes' jobs: packed board words 0..6, player | d0 << 8 | d1 << 16
    LaneState st[FL];               // the lanes' state for the whole launch (written back at the end)
};
template <int FL> struct FCfg {
    static constexpr int NW = FL == 32 ? BGX_FUSED_NW32 : BGX_FUSED_NW16;
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
    // V(s), V(candidates 0..XS-2) of each lane kept in LDS (the rest: vbuf): as many as fit (<= 96)
    static constexpr int XS_FIT = (160 * 1024 - F_TAIL - (int)sizeof(FusedTail<FL>)) / (FL * 4);
    static constexpr int XS = XS_FIT < 96 ? XS_FIT : 96;
    static constexpr int LDS = F_TAIL + (int)sizeof(FusedTail<FL>) + FL * XS * 4;
    static_assert(XS >= 24 && LDS <= 160 * 1024, "fits the CU's LDS");
};

template <bool PROF, int FL>
__global__ __launch_bounds__(64 * FCfg<FL>::NW, FCfg<FL>::WPE) void fused_step_kernel(FusedArgs f) {
    using C = FCfg<FL>;
    constexpr int NW = C::NW, SL1 = C::SL1, F_W = C::F_W, F_TAIL = C::F_TAIL, XS = C::XS;
    constexpr int P1_S = C::P1_S, P1_F = C::P1_F, P1_PF = C::P1_PF;
    constexpr int CP_F = C::CP_F;
    // the cooperative tier 2 at 12 waves only (at 8 waves, 256 registers, its
    // registers spill in the step loop: 0 -> 19)
    constexpr bool COOP2 = NW > 8;
    constexpr int NT = 64 * NW;          // threads
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    uint8_t* lds = (uint8_t*)smem;
    FusedTail<FL>& T = *(FusedTail<FL>*)(lds + F_TAIL);
    float* xs = (float*)(lds + F_TAIL + sizeof(FusedTail<FL>));   // [FL][XS] lane values
    const EngineDev& e = f.e;
    const int t = (int)threadIdx.x, w = t >> 6, l = lane_id();
    for (int i = t; i < 256; i += NT) T.lut[i] = lut_entry((uint32_t)i, f.feat_scale);
    for (int i = t; i < 128; i += NT) T.w2s[i] = f.rowc[i];
    for (int i = t; i < 64; i += NT) T.tdone[i] = 0u;
    for (int i = t; i < FL; i += NT) T.chosen[i] = T.claim[i] = 0u;
    unsigned qtag = 0u;   // this workgroup's step counter (tags the flags; never 0 on a live step)
    int half_b = 0;       // thread 0: the half a half-lane ticket steps next (ticket)
    // split-fp16 W fragments, loaded once, global -> LDS by LDS-DMA (every load
    // of a wave in flight at once; the prologue's lane loads overlap them)
    uint4* wl = (uint4*)(lds + F_W);
    static_assert(NFRAG % 64 == 0, "W fragments in whole wave chunks");
    for (int c = w; c < NFRAG / 64; c += NW)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(void*)(f.wfrag + 64 * c + l),
                                         (__attribute__((address_space(3))) void*)(void*)(wl + 64 * c), 16, 0, 0);
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
    const unsigned long long cyc_begin = PROF ? __builtin_amdgcn_s_memtime() : 0ull;   // shader clock (f.prof)
    unsigned long long t_loop0 = 0, t_loop1 = 0;   // first step's start, last step's end (f.prof)
    // step durations by index within the launch (f.prof): steps 0..23 go to
    // P[32 + k] (their count to P[64 + k]) as they end, later ones are summed here
    unsigned long long t_step = 0, late_sum = 0, late_n = 0;
    int step_idx = 0;
    // development timers (f.prof): phase sums on thread 0, per-wave sums on lane 0
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tc = 0, tw[4] = {0, 0, 0, 0}, t2c = 0, t3n = 0;
    unsigned long long tjd[4] = {0, 0, 0, 0};   // tier-1 job clocks / counts: doubles, non-doubles
    unsigned long long tcs[3] = {0, 0, 0};      // choice: state + Philox refill, pick, env step (lane_advance)
    unsigned long long tms[3] = {0, 0, 0};      // MLP tile: rows + k mask, MFMA chain issue, drain + epilogue
    constexpr bool prof = PROF;
    auto tick = [&](int k) {
        if (prof && t == 0) {
            const unsigned long long c = wall_clock64();
            ph[k] += c - tc;
            tc = c;
        }
    };
    // ---------------------------------------------------------------- pipelined steps
    // Step s is one LDS item queue: its MLP tiles, then its choice items (a pair
    // of lanes each), then the next step's tier-1 jobs (one lane each). A choice
    // item waits (LDS flags, bounded) for the tiles holding its lanes' rows; a
    // tier-1 job waits for its lane's choice. Every item a waiting item needs
    // is handed out before it, and tiles wait on nothing, so the waits end.
    // The MFMA-bound tiles, the latency-bound choice chains and the issue-bound
    // tier-1 jobs then share the SIMDs instead of running in barrier-separated
    // phases; the barriers left per step are the ones around the workgroup
    // tiers (tier 2) and the row prefix. The tiles read their rows from the
    // candidate buffer (L2) rather than from a staged copy in the scratch, which
    // holds the waves' tier-1 slices during the queue.
    const int groups = (e.L + FL - 1) / FL;
    uint32_t* const slw = (uint32_t*)(lds + (size_t)w * SL1);   // this wave's tier-1 slice
    Mem M1;
    M1.map = slw;
    M1.tab = (unsigned long long*)(slw + 64);
    M1.S = P1_S;
    M1.F = P1_F;
    M1.fa = slw + 64 + 2 * P1_S;
    M1.fb = M1.fa + P1_F;
    M1.pa = slw + 64;
    M1.pb = M1.pa + P1_PF;
    M1.PF = P1_PF;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's W fragment loads landed (a barrier follows)
    for (int g = (int)blockIdx.x; g < groups; g += (int)gridDim.x) {
        const int nlive = e.L - g * FL < FL ? e.L - g * FL : FL;
        for (int v = t; v < nlive; v += NT) {
            lane_load(e, g * FL + v, T.st[v]);
            if (f.t1_ready) T.cnt[v] = f.t1cnt[g * FL + v];   // the previous launch expanded these positions
        }
        if (f.t1_ready) {   // the jobs' words for tier 2 (T.job), from the lane states
            __syncthreads();
            for (int q = t; q < nlive * 8; q += NT) {
                const int v = q >> 3, k = q & 7;
                const LaneState& st = T.st[v];
                T.job[v][k] = k < 7 ? st.w[k] : (uint32_t)st.p | ((uint32_t)st.d0 << 8) | ((uint32_t)st.d1 << 16);
            }
        }
        // step s runs iff ticket(s): lockstep, s < n_steps; balanced, s < n_cap and
        // the launch's lane-step total before this workgroup-step is below the
        // budget (thread 0 takes step s + 1's ticket after step s's queue, which
        // expanded the next positions whatever the ticket says: a refused ticket
        // ends the launch with them ready for the next one)
        // A ticket is the step's lane range, lo | hi << 8 (0: stop). In the
        // launch's last round (less than one full step of every workgroup left in
        // the budget) a balanced workgroup steps half its lanes at a time, the two
        // halves in turn: a half step is ~0.6 of a full one, so the workgroups'
        // ends, spread over the step that each was in when the budget ran out,
        // lie closer together. Each lane's game is its own (dice and uniforms are
        // keyed by lane and its counter), so which lanes step when changes nothing
        // but how far each lane has got at a harvest.
        auto ticket = [&](int s) -> int {
            const int full = nlive << 8;
            if (f.budget <= 0) return s < f.n_steps ? full : 0;
            if (s >= f.n_cap) return 0;
            int lo = 0, hi = nlive;
            if (BGX_HALF_TICKETS && nlive >= 2) {
                const long long left =
                    f.budget - (long long)__hip_atomic_load(f.budget_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (left < (long long)gridDim.x * (long long)nlive) {
                    half_b ^= 1;
                    lo = half_b ? nlive >> 1 : 0;
                    hi = half_b ? nlive : nlive >> 1;
                }
            }
            const unsigned long long old = atomicAdd(f.budget_ctr, (unsigned long long)(hi - lo));
            return old < (unsigned long long)f.budget ? lo | (hi << 8) : 0;
        };
        // bounded wait for an LDS flag
        auto wait_flag = [&](const unsigned* fl) {
            for (unsigned spin = 0; __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != qtag;
                 ++spin) {
                if (spin >= (1u << 24)) {
                    if (l == 0) atomicOr(e.err_flags, BGX_ERRF_WAIT_BOUND);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        };
        const int n_iter = f.budget > 0 ? f.n_cap : f.n_steps;
        if (prof && t == 0 && !t_loop0) t_loop0 = wall_clock64();
        // step -1 is the first step's tier-1 queue alone; step s >= 0: tier 2 and
        // the row prefix of step s, then its queue (tiles, choice pairs, step
        // s + 1's tier-1 jobs). Each item kind is issued from one place in the
        // code (the kernel is at its register cap: the movegen and MLP bodies are
        // inlined once each).
        for (int step = -1; step < n_iter; ++step) {
            int nr = 0;
            // this step's lanes [lo, hi) (step -1, the first step's tier-1 jobs: all)
            const int gv = step >= 0 ? T.go[step & 1] : nlive << 8;
            if (!gv) break;
            const int lo = gv & 255, hi = gv >> 8;
            const auto act = [&](int v) { return v >= lo && v < hi; };
            if (prof && t == 0) tc = wall_clock64();
            if (step >= 0) {
                n_steps += (unsigned long long)(hi - lo);
                // ---- 1b. jobs that outgrew their slice: the workgroup, one at a time (rare)
                const int cnt_l = act(l) ? T.cnt[l] : 0;   // lane q < FL holds lane q's count
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
                // computes it (identical values)
                const int c = act(l) ? T.cnt[l] : 0;   // lanes outside this step's range: no rows
                const int rows = l < FL && c > 0 ? 1 + (c < f.cap ? c : f.cap) : 0;
                const int incl = wave_incl_scan(rows);
                if (l <= FL) T.pre[l] = incl - rows;
                wave_sync();
                nr = T.pre[FL];
                n_rows += (unsigned long long)nr;
                tick(1);
            }
            const int n_tiles = (nr + 31) >> 5;
            const int np = step >= 0 ? (hi - lo + 1) >> 1 : 0;   // choice items: lane pairs
            if (t == 0) {
                T.qn[0] = NW;
                T.qn[1] = NW;
            }
            ++qtag;
            M1.map[l] = 0u;   // (tier 2 may have used the scratch)
            wave_sync();
            __syncthreads();
            // step s + 1's tier-1 jobs (every step: the last one's results are
            // the next launch's first; at step -1, unless the previous launch
            // left them)
            const int nj = step >= 0 || !f.t1_ready ? hi - lo : 0;
            // the next step's jobs, doubles first, when nothing runs beside them
            const bool dbl = act(l) && T.st[l].d0 == T.st[l].d1;
            const uint32_t dmask = (uint32_t)ballot(dbl), omask = (uint32_t)ballot(act(l) && !dbl);
            const int nd = __popc(dmask);
            // row r of the workgroup -> its lane: the last v with pre[v] <= r
            auto lane_of = [&](int r) -> int {
                int v = 0;
#pragma unroll
                for (int sstep = FL / 2; sstep >= 1; sstep >>= 1)
                    if (T.pre[v + sstep] <= r) v += sstep;
                return v;
            };
            const unsigned long long m0 = prof ? wall_clock64() : 0ull;
            // one pass when the tile flags cover the step (the usual case), else
            // tiles, choices and jobs in three barrier-separated passes
            const bool one = n_tiles <= 64;
            const int npass = one ? 1 : 3;
            for (int pass = 0; pass < npass; ++pass) {
                const int qt = one || pass == 0 ? n_tiles : 0;
                const int qp = one || pass == 1 ? np : 0;
                const int qj = one || pass == 2 ? nj : 0;
                const bool pipelined = one && np > 0;   // waits between items of the same queue
                int* qc = &T.qn[pass & 1];
                int it = w;
                while (it < qt + qp + qj) {
                    if (it < qt) {
                        // ---- 3. one MLP tile: its 32 rows from the lanes' obs rows /
                        // candidate slots (L2), all four m-tiles in the wave (mlp_tile4)
                        const unsigned long long i0 = prof ? wall_clock64() : 0ull;
                        const int r = it * 32 + (l & 31);
                        uint4 bx = make_uint4(0, 0, 0, 0), by = make_uint4(0, 0, 0, 0);
                        int vl = 0, k = 0;
                        if (r < nr) {
                            vl = lane_of(r);
                            k = r - T.pre[vl];
                            const int li = g * FL + vl;
                            const uint32_t* src =
                                k == 0 ? e.rows + (size_t)li * 8 : f.cand + ((size_t)li * f.cap + (k - 1)) * 8;
                            bx = ((const uint4*)src)[0];
                            by = ((const uint4*)src)[1];
                        }
                        const uint32_t km = tile_kmask(bx, by);
                        unsigned long long i1 = 0, i2 = 0;
                        if (prof) {
                            __builtin_amdgcn_s_waitcnt(0);
                            i1 = wall_clock64();
                            tms[0] += i1 - i0;   // rows loaded, lane_of, k mask
                        }
                        const float v = mlp_tile4<PROF>(wf, T.lut, T.w2s, f.feat_scale, bx, by, km, &i2);
                        if (prof) {
                            const float vv = __shfl(v, 0);   // the epilogue's value is ready
                            asm volatile("" ::"v"(vv));
                            const unsigned long long i3 = wall_clock64();
                            tms[1] += i2 - i1;   // MFMA chain issued
                            tms[2] += i3 - i2;   // drain + epilogue
                        }
                        if (l < 32 && r < nr) {
                            const float val = v + f.b2;
                            if (k < XS) xs[vl * XS + k] = val;
                            else f.vbuf[(size_t)(g * FL + vl) * (f.cap + 1) + k] = val;
                        }
                        // the tile's values (LDS and, past XS, vbuf) before its flag
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (l == 0) __hip_atomic_store(&T.tdone[it & 63], qtag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (prof) tw[1] += wall_clock64() - i0;
                    } else if (it < qt + qp) {
                        // ---- 4. action choice + env step of two lanes, one per half-wave
                        const int p = it - qt;
                        if (pipelined) {
                            const int va = lo + 2 * p, vb = lo + 2 * p + 2 < hi ? lo + 2 * p + 2 : hi;
                            const int r0 = T.pre[va], r1 = T.pre[vb];   // the pair's rows [r0, r1)
                            if (r1 > r0) {
                                for (int tt = r0 >> 5; tt <= (r1 - 1) >> 5; ++tt) wait_flag(&T.tdone[tt]);
                                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                            }
                        }
                        const int v = lo + 2 * p + (l >> 5);
                        const bool lead = (l & 31) == 0;
                        if (v < hi) {
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
                                        ? pick_action_half([&](int kk) { return xv[1 + kk] / Tm; }, n, e.greedy != 0, u)
                                        : pick_action_half(
                                              [&](int kk) { return (1 + kk < XS ? xv[1 + kk] : vv[1 + kk]) / Tm; }, n,
                                              e.greedy != 0, u);
                                if (prof) {
                                    const unsigned long long c1 = wall_clock64();
                                    tw[2] += c1 - s1;
                                    tcs[1] += c1 - c0;
                                    c0 = c1;
                                }
                                uint32_t nb[8];
                                load_packed(f.cand + ((size_t)i * f.cap + pick) * 8, nb);
                                const float va = 1 + pick < XS ? xv[1 + pick] : vv[1 + pick];
                                lane_advance(e, i, sr, rng, pick, nb, xv[0], va, n_full, lead);
                                if (prof) {
                                    __builtin_amdgcn_s_waitcnt(0);
                                    tcs[2] += wall_clock64() - c0;
                                }
                            }
                            wave_sync();
                            if (lead) T.st[v] = sr;
                            if (prof) tw[3] += wall_clock64() - s1;
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (lead && v < hi)
                            __hip_atomic_store(&T.chosen[v], qtag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        // ---- 1. a tier-1 job of the next step in this wave's slice:
                        // lane order behind the choices (a lane's job waits for its
                        // choice), doubles first when the queue holds jobs only
                        const int kj = it - qt - qp;
                        int v;
                        if (pipelined) {
                            // the first stepped and unclaimed lane, doubles (the long
                            // jobs) first; every job item claims one lane, and every
                            // lane's choice was handed out before any job item
                            v = -1;
                            for (unsigned spin = 0; v < 0; ++spin) {
                                const bool ready =
                                    act(l) &&
                                    __hip_atomic_load(&T.chosen[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == qtag &&
                                    __hip_atomic_load(&T.claim[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != qtag;
                                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                                const bool isd = ready && T.st[l].d0 == T.st[l].d1;
                                const uint32_t md = (uint32_t)ballot(isd), mo = (uint32_t)ballot(ready && !isd);
                                if (md | mo) {
                                    const int cand = md ? __ffs(md) - 1 : __ffs(mo) - 1;
                                    int won = 0;
                                    if (l == 0) {
                                        const unsigned old = T.claim[cand];
                                        won = old != qtag && atomicCAS(&T.claim[cand], old, qtag) == old;
                                    }
                                    if (uniform(won)) v = cand;
                                } else {
                                    if (spin >= (1u << 24)) {   // bounded
                                        if (l == 0) atomicOr(e.err_flags, BGX_ERRF_WAIT_BOUND);
                                        v = kj;
                                        break;
                                    }
                                    __builtin_amdgcn_s_sleep(1);
                                }
                            }
                        } else {
                            v = kj < nd ? select_bit(dmask, kj) : select_bit(omask, kj - nd);
                        }
                        const unsigned long long q0 = prof ? wall_clock64() : 0ull;
                        const LaneState& st = T.st[v];
                        if (l < 8)
                            T.job[v][l] = l < 7 ? st.w[l] : (uint32_t)st.p | ((uint32_t)st.d0 << 8) | ((uint32_t)st.d1 << 16);
                        const JobIn in =
                            make_job(st.w[0], st.w[1], st.w[2], st.w[3], st.w[4], st.w[5], st.w[6], st.p, st.d0, st.d1);
#if BGX_FUSED_LEAF
                        // path doubles stream their leaves past the slice's list (no tier 2)
                        FlatCursor fcj;
                        const int nf = f.force_tier >= 2 ? -1 : run_job<false, true>(a, g * FL + v, in, M1, fcj);
#else
                        uint32_t* fin = nullptr;
                        const int nf = f.force_tier >= 2 ? -1 : job_records<false>(in, M1, fin, 0x7FFFFFFF);
                        if (nf >= 0) emit_records<false>(a, g * FL + v, in, fin, nf, 0);
#endif
                        wave_sync();
                        if (l == 0) T.cnt[v] = nf;
                        if (prof) {
                            const int kd = in.d0 == in.d1 ? 0 : 2;
                            tjd[kd] += wall_clock64() - q0;
                            tjd[kd + 1] += 1;
                        }
                    }
                    int kn = 0;
                    if (l == 0) kn = atomicAdd(qc, 1);
                    it = uniform(kn);
                }
                if (pass + 1 < npass) {
                    if (t == 0) T.qn[(pass + 1) & 1] = NW;   // (the next pass's counter, unused since its reset)
                    __syncthreads();
                }
            }
            if (prof) tw[0] += wall_clock64() - m0;
            tick(3);
            if (t == 0) T.go[(step + 1) & 1] = ticket(step + 1);   // as late as the step allows
            __syncthreads();   // step s's lanes are stepped and step s + 1's jobs are done
            tick(4);
            if (prof && t == 0 && step >= 0) ph[5] += 1;
            if (prof && t == 0) {
                const unsigned long long c = wall_clock64();
                if (step >= 0) {
                    if (step_idx < 24) {
                        atomicAdd(f.prof + (size_t)blockIdx.x * PROF_STRIDE + 32 + step_idx, c - t_step);
                        atomicAdd(f.prof + (size_t)blockIdx.x * PROF_STRIDE + 64 + step_idx, 1ull);
                    }
                    else { late_sum += c - t_step; ++late_n; }
                    ++step_idx;
                }
                t_step = c;
            }
        }
        if (prof && t == 0) t_loop1 = wall_clock64();
        for (int v = t; v < nlive; v += NT) {
            lane_store(e, g * FL + v, T.st[v]);
            f.t1cnt[g * FL + v] = T.cnt[v];   // the next positions' expansion (f.t1_ready)
        }
        if (f.hv_hdr) {
            // ---- in-kernel harvest: this group's finished episodes (headers from
            // the lanes' header rings, records from their record rings) appended to
            // the ticket's output at offsets from one 64-bit atomic, while other
            // workgroups still run their last steps (the scratch is free here)
            uint32_t* hs = (uint32_t*)lds;   // [0, 64) episode prefix, [64, 128) record prefix, [128, 133) totals
            if (w == 0) {
                int ne = 0, nr = 0;
                bool lost = false;
                if (l < nlive) {
                    const LaneState& s = T.st[l];
                    ne = (int)(s.epi - s.hepi);
                    nr = (int)(s.ep_first - s.harv);
                    // past its header ring or record ring (flagged when it happened):
                    // this lane's finished episodes are gone; only it is left out
                    lost = ne > e.HR || nr > e.R;
                }
                if (lost) ne = nr = 0;
                const int ie = wave_incl_scan(ne), ir = wave_incl_scan(nr);
                const uint32_t te = (uint32_t)__shfl(ie, 63), tr = (uint32_t)__shfl(ir, 63);
                if (l < FL) {
                    hs[l] = (uint32_t)(ie - ne);
                    hs[64 + l] = (uint32_t)(ir - nr);
                }
                if (l == 0) {
                    // the group's place in the ticket's output: one fetch-add of its
                    // totals on the reservation counter (a compare-and-swap loop here
                    // serialised the 256 workgroups that finish together: +0.24 ms per
                    // launch). A group whose range ends past the output's capacity
                    // (several launches between two tickets append to one output)
                    // copies nothing and keeps its episodes in the rings for the next
                    // ticket; every group reserved after it starts past the capacity
                    // too, so the groups that fit are a prefix of the reservations and
                    // their sum (the commit counter) is the ticket's contiguous total
                    unsigned long long base = 0ull;
                    uint32_t fit = 1u;
                    if (te | tr) {
                        const unsigned long long add = ((unsigned long long)te << 32) | tr;
                        base = atomicAdd(f.hv_ctr, add);
                        fit = (base >> 32) + te <= (unsigned long long)f.hv_ep_cap &&
                              (base & 0xFFFFFFFFull) + tr <= (unsigned long long)f.hv_rec_cap;
                        if (fit) atomicAdd(f.hv_commit, add);
                    }
                    hs[128] = te;
                    hs[129] = tr;
                    hs[130] = (uint32_t)(base >> 32);
                    hs[131] = (uint32_t)base;
                    hs[132] = fit;
                }
                if (l < FL) hs[136 + l] = lost ? 1u : 0u;
            }
            __syncthreads();
            const uint32_t te = hs[128], tr = hs[129], be = hs[130], br = hs[131], fit = hs[132];
            // lane of the k-th episode / record: the last v with prefix[v] <= k
            auto owner = [&](const uint32_t* pre, uint32_t k) -> int {
                int v = 0;
#pragma unroll
                for (int sstep = FL / 2; sstep >= 1; sstep >>= 1)
                    if (pre[v + sstep] <= k) v += sstep;
                return v;
            };
            if (fit) {
                for (uint32_t q = (uint32_t)t; q < 4u * te; q += NT) {   // 4 x uint4 per header
                    const uint32_t k = q >> 2;
                    const int v = owner(hs, k);
                    const uint32_t ep = T.st[v].hepi + (k - hs[v]);
                    const uint4* src = (const uint4*)(e.hring + ((size_t)(g * FL + v) * e.HR + (ep & (uint32_t)(e.HR - 1))) *
                                                                    EP_WORDS);
                    ((uint4*)(f.hv_hdr + (size_t)(be + k) * EP_WORDS))[q & 3u] = src[q & 3u];
                }
                for (uint32_t q = (uint32_t)t; q < 3u * tr; q += NT) {   // 3 x uint4 per record
                    const uint32_t r = q / 3u, c = q - 3u * r;
                    const int v = owner(hs + 64, r);
                    const uint32_t rr = T.st[v].harv + (r - hs[64 + v]);
                    const uint4* src =
                        (const uint4*)(e.ring + ((size_t)(g * FL + v) * e.R + (rr & (uint32_t)(e.R - 1))) * REC_WORDS);
                    ((uint4*)(f.hv_rec + (size_t)(br + r) * REC_WORDS))[c] = src[c];
                }
            }
            for (int v = t; v < nlive; v += NT) {
                if (fit || hs[136 + v]) {   // harvested (or lost): the marks move on
                    e.harv[g * FL + v] = T.st[v].ep_first;
                    e.hepi[g * FL + v] = T.st[v].epi;
                }
            }
        }
        __syncthreads();
    }
    if (prof) {
        unsigned long long* P = f.prof + (size_t)blockIdx.x * PROF_STRIDE;
        if (t == 0) {
            // the last launch's begin / end clocks, rows and tier-2 jobs of this
            // workgroup (overwritten per launch: the spread of the workgroups'
            // durations is what a short launch waits for)
            P[24] = wg_begin;
            P[25] = wall_clock64();
            P[26] = n_rows;
            P[27] = n_fb;
            P[28] = n_steps;
            P[19] = t_loop0;
            P[20] = t_loop1;
            P[21] = __builtin_amdgcn_s_memtime() - cyc_begin;
            for (int k = 0; k < 6; ++k) atomicAdd(P + k, ph[k]);
            atomicAdd(P + 11, t2c);
            atomicAdd(P + 12, n_fb);
            atomicAdd(P + 13, t3n);
            atomicAdd(P + 18, (unsigned long long)NW * ph[5]);   // wave-steps
            atomicAdd(P + 56, late_sum);
            atomicAdd(P + 57, late_n);
        }
        if (l == 0) {
            for (int k = 0; k < 4; ++k) atomicAdd(P + 7 + k, tw[k]);
            for (int k = 0; k < 4; ++k) atomicAdd(P + 14 + k, tjd[k]);
            for (int k = 0; k < 3; ++k) atomicAdd(P + 29 + k, tcs[k]);
            atomicAdd(P + 6, tms[0]);
            atomicAdd(P + 22, tms[1]);
            atomicAdd(P + 23, tms[2]);
        }
    }
    if (t == 0) {
        atomicAdd(e.stats + 0, n_steps);
        atomicAdd(e.stats + 3, n_rows);
        atomicAdd(e.stats + 4, n_steps);
        atomicAdd(e.stats + 5, n_fb);
        if (f.budget > 0 || f.hv_hdr) {
            // the last workgroup to finish zeroes the lane-step counter for the
            // next launch and publishes the harvest totals (stream order: no
            // memset or harvest launch in between)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (atomicAdd(f.done_ctr, 1ull) == (unsigned long long)gridDim.x - 1ull) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (f.budget > 0) __hip_atomic_store(f.budget_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (f.hv_hdr) {
                    const unsigned long long c = __hip_atomic_load(f.hv_commit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    // the launch's flags move into this ticket's accumulator (stream
                    // order: the fetch never resets the engine word behind a launch)
                    const uint32_t fl = atomicExch(e.err_flags, 0u) | (uint32_t)*f.hv_flags;
                    *f.hv_flags = fl;
                    *f.hv_next_flags = 0ull;
                    const uint32_t v[4] = {(uint32_t)(c >> 32), (uint32_t)c, fl, (uint32_t)(c >> 32)};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        f.hv_info[k] = v[k];
                        if (f.hv_hinfo) f.hv_hinfo[k] = v[k];   // host-mapped (vector stores)
                    }
                    __hip_atomic_store(f.hv_next, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(f.hv_next_commit, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(f.done_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    // per device (one process may drive several GPUs: multi/worker.py gives
    // worker 0 GPUs 0 and 7): the CU count and the kernels' dynamic-LDS opt-in
    static int n_cu_dev[64] = {0};
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur < 0 || cur >= 64) cur = 0;
    int& n_cu = n_cu_dev[cur];
    if (!n_cu) {
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, cur) != hipSuccess || n_cu <= 0)
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
