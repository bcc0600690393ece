// bgx_fused.hip — the 1-ply self-play step fused into one persistent launch.
//
// One workgroup of 16 wavefronts owns 16 game lanes (one lane per wave) and
// runs n_steps env steps of each, with no kernel boundary between the steps:
//   1. movegen: each wave expands its lane's (board, player, dice) job in its
//      own 8 KB LDS slice (tier 1, bgx_movegen.h) and writes the afterstates to
//      the lane's candidate slots; a job that outgrows the slice is redone by
//      the whole workgroup after the barrier (cooperative doubles / 32 KB
//      slice / global workspace: the movegen_block_kernel tiers);
//   2. the LDS that held the slices now takes the split-fp16 W fragments;
//   3. value MLP over the workgroup's rows (the lanes' obs rows + candidates,
//      ~350 per step) in 32-board MFMA tiles spread over the 16 waves
//      (mlp_item: one (tile, m-tile) per wave at a time, partials summed in the
//      canonical order, so V has the same bits as the phased engine's);
//   4. each wave samples its lane's action from softmax(V/T) and lane 0 runs
//      the env step (lane_advance: apply, rewards, record, reset) on the
//      lane's state, which stays in the wave's registers for the whole launch.
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

constexpr int FW = BW;                                  // waves = lanes per workgroup (16)
constexpr int F_OVL = FW * Slice<S_T1>::bytes;          // overlay: slices | CoopLds | W | select scratch
static_assert(sizeof(CoopLds) <= (size_t)F_OVL, "cooperative tier fits the overlay");
static_assert(NFRAG * 16 <= F_OVL, "W fragments fit the overlay");
static_assert(Slice<S_T2>::bytes <= F_OVL, "32 KB slice fits the overlay");

struct FusedTail {
    uint4 lut[256];                 // feature LUT (bgx_mlp.h lut_entry)
    float w2s[128];                 // value-head weights
    int cnt[FW];                    // lane's full candidate count this step (-1: redo in tier 2)
    int pre[FW + 1];                // MLP row prefix over the lanes
    uint32_t job[FW][8];            // the lanes' jobs: packed board words 0..6, player | d0 << 8 | d1 << 16
    LaneState st[FW];               // the lanes' state for the whole launch (written back at the end)
};
constexpr int F_LDS = F_OVL + (int)sizeof(FusedTail);
constexpr int FT = (F_OVL - NFRAG * 16) / (4 * 64 * 4 + 32 * 32);   // MLP tiles per batch: partials + rows after W
static_assert(FT >= 4, "partials fit behind W");

template <bool PROF>
__global__ __launch_bounds__(64 * FW) void fused_step_kernel(FusedArgs f) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    uint8_t* lds = (uint8_t*)smem;
    FusedTail& T = *(FusedTail*)(lds + F_OVL);
    const EngineDev& e = f.e;
    const int t = (int)threadIdx.x, w = t >> 6, l = lane_id();
    for (int i = t; i < 256; i += 64 * FW) T.lut[i] = lut_entry((uint32_t)i, f.feat_scale);
    for (int i = t; i < 128; i += 64 * FW) T.w2s[i] = f.rowc[i];

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
    // development timers (f.prof): phase sums on thread 0, tier-1 job time per wave
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tj = 0, tc = 0, tw[4] = {0, 0, 0, 0};
    constexpr bool prof = PROF;
    auto tick = [&](int k) {
        if (prof && t == 0) {
            const unsigned long long c = wall_clock64();
            ph[k] += c - tc;
            tc = c;
        }
    };
    const int groups = (e.L + FW - 1) / FW;
    for (int g = (int)blockIdx.x; g < groups; g += (int)gridDim.x) {
        const int i = g * FW + w;   // this wave's lane
        const bool live = i < e.L;
        // the lane's state stays in LDS for all n_steps (every lane of the wave
        // computes the same update; lane 0 writes memory)
        LaneState& st = T.st[w];
        if (live) lane_load(e, i, st);
        n_steps += (unsigned long long)(e.L - g * FW < FW ? e.L - g * FW : FW) * (unsigned long long)f.n_steps;
        for (int step = 0; step < f.n_steps; ++step) {
            // ---- 1. tier-1 movegen in the wave's slice
            if (prof && t == 0) tc = wall_clock64();
            {
                const unsigned long long j0 = prof ? wall_clock64() : 0ull;
                unsigned long long* sl = smem + (size_t)w * (Slice<S_T1>::bytes / 8);
                Mem M;
                M.tab = sl;
                M.F = Slice<S_T1>::F;
                M.fa = (uint32_t*)(sl + S_T1);
                M.fb = M.fa + M.F;
                M.map = M.fb + M.F;
                M.S = S_T1;
                M.map[l] = 0u;
                wave_sync();
                int nf = 0;
                if (live) {
                    if (l < 8)
                        T.job[w][l] = l < 7 ? st.w[l] : (uint32_t)st.p | ((uint32_t)st.d0 << 8) | ((uint32_t)st.d1 << 16);
                    const JobIn in = make_job(st.w[0], st.w[1], st.w[2], st.w[3], st.w[4], st.w[5], st.w[6], st.p,
                                              st.d0, st.d1);
                    uint32_t* fin = nullptr;
                    nf = f.force_tier >= 2 ? -1 : job_records<false>(in, M, fin, 0x7FFFFFFF);
                    if (nf >= 0) emit_records<false>(a, i, in, fin, nf, 0);
                }
                if (l == 0) T.cnt[w] = nf;
                if (prof) tj += wall_clock64() - j0;
            }
            __syncthreads();
            tick(0);
            // ---- 1b. jobs that outgrew their slice: the whole workgroup, one at a time
            for (int v = 0; v < FW; ++v) {
                if (T.cnt[v] >= 0) continue;   // uniform: LDS after a barrier
                ++n_fb;
                const int j = g * FW + v;
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
                    const int r = run_job<true>(a, j, in, G, fc);
                    if (r < 0 && l == 0) atomicOr(e.err_flags, BGX_ERRF_FALLBACK_OVERFLOW);
                    return r < 0 ? 0 : r;
                };
                if (in.d0 != in.d1 || f.force_tier >= 3) {
                    if (w == 0) {
                        const Mem M2 = lds_mem<S_T2>(smem);
                        int r = f.force_tier >= 3 ? -1 : run_job<false>(a, j, in, M2, fc);
                        if (r < 0) r = run_global();
                        if (l == 0) T.cnt[v] = r;
                    }
                } else {
                    CoopLds& C = *(CoopLds*)smem;
                    uint32_t* fin = nullptr;
                    const int nfin = coop_doubles(in, C, fin);   // block-uniform
                    if (nfin >= 0) {
                        for (int k = t; k < nfin && k < f.cap; k += 64 * FW) {
                            const uint32_t x = fin[k];
                            emit_one(a, j, in.R,
                                     (x & PATHF) ? path_board(in.R, x & KEYMASK, in.d0)
                                                 : rebuild(in.R, x & KEYMASK, in.d0),
                                     k, 0);
                        }
                        if (t == 0) T.cnt[v] = nfin;
                    } else if (w == 0) {
                        const int r = run_global();
                        if (l == 0) T.cnt[v] = r;
                    }
                }
                __syncthreads();
            }
            tick(1);
            // ---- 2. row prefix (lanes that pass evaluate nothing) + W fragments into the overlay
            if (t == 0) {
                int acc = 0;
                for (int v = 0; v < FW; ++v) {
                    T.pre[v] = acc;
                    const int c = T.cnt[v];
                    acc += c > 0 ? 1 + (c < f.cap ? c : f.cap) : 0;
                }
                T.pre[FW] = acc;
            }
            uint4* wf = (uint4*)lds;
            for (int k = t; k < NFRAG; k += 64 * FW) wf[k] = f.wfrag[k];
            __syncthreads();
            tick(2);
            // ---- 3. value MLP over the workgroup's rows: (32-board tile, m-tile)
            // items spread over the 16 waves, partials combined in the
            // canonical epilogue order (bgx_mlp.h); batches of FT tiles
            const int nr = T.pre[FW];
            n_rows += (unsigned long long)nr;
            const unsigned long long m0 = prof ? wall_clock64() : 0ull;
            // row r of the workgroup -> its packed board / its V slot
            auto lane_of = [&](int r) -> int {
                int v = 0;
#pragma unroll
                for (int q = 1; q < FW; ++q) v += T.pre[q] <= r ? 1 : 0;
                return v;
            };
            auto row_of = [&](int r, uint4& bx, uint4& by) {
                const int v = lane_of(r), k = r - T.pre[v];
                const int li = g * FW + v;
                const uint32_t* src =
                    k == 0 ? e.rows + (size_t)li * 8 : f.cand + ((size_t)li * f.cap + (k - 1)) * 8;
                bx = ((const uint4*)src)[0];
                by = ((const uint4*)src)[1];
            };
            auto vslot = [&](int r) -> size_t {
                const int v = lane_of(r), k = r - T.pre[v];
                return (size_t)(g * FW + v) * (f.cap + 1) + k;
            };
            // batch of FT tiles: rows staged in LDS (one global load per row, all
            // in flight together), then the items, then the combine
            float* vp = (float*)(lds + NFRAG * 16);                 // [4][FT][64] partials
            uint4* rs = (uint4*)(lds + NFRAG * 16 + 4 * FT * 64 * 4);   // [FT * 32][2] staged rows
            const int n_tiles = (nr + 31) >> 5;
            for (int tb = 0; tb < n_tiles; tb += FT) {
                const int nt = n_tiles - tb < FT ? n_tiles - tb : FT;
                if (tb > 0) __syncthreads();   // the previous batch's rows / partials are consumed
                for (int c = t; c < nt * 32; c += 64 * FW) {
                    const int r = tb * 32 + c;
                    uint4 bx = make_uint4(0, 0, 0, 0), by = make_uint4(0, 0, 0, 0);
                    if (r < nr) row_of(r, bx, by);
                    rs[2 * c] = bx;
                    rs[2 * c + 1] = by;
                }
                __syncthreads();
                for (int it = w; it < 4 * nt; it += FW) {
                    const int tl = it >> 2, m = it & 3;
                    const int c = tl * 32 + (l & 31);
                    const uint4 bx = rs[2 * c], by = rs[2 * c + 1];
                    vp[(m * FT + tl) * 64 + l] =
                        mlp_item(wf, T.lut, T.w2s, f.feat_scale, bx, by, tile_kmask(bx, by), m);
                }
                __syncthreads();
                for (int c = t; c < nt * 32; c += 64 * FW) {
                    const int tl = c >> 5, col = c & 31;
                    const int r = (tb + tl) * 32 + col;
                    if (r < nr) {
                        float vh[2];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int q = tl * 64 + col + 32 * h;
                            vh[h] = ((vp[q] + vp[FT * 64 + q]) + vp[2 * FT * 64 + q]) + vp[3 * FT * 64 + q];
                        }
                        f.vbuf[vslot(r)] = (vh[0] + vh[1]) + f.b2;
                    }
                }
            }
            if (prof) tw[0] += wall_clock64() - m0;
            __syncthreads();
            tick(3);
            // ---- 4. action choice + env step (the overlay is free again: scratch)
            if (live) {
                const int n_full = T.cnt[w];
                const int n = n_full < e.max_legal ? n_full : e.max_legal;
                if (n <= 0) {
                    lane_advance(e, i, st, -1, e.rows + (size_t)i * 8, 0.0f, 0.0f, 0, l == 0);
                } else {
                    float* x = (float*)lds + (size_t)w * (F_OVL / 4 / FW);
                    const float* vv = f.vbuf + (size_t)i * (f.cap + 1);
                    const float Tm = e.temperature;
                    const unsigned long long s0 = prof ? wall_clock64() : 0ull;
                    for (int k = l; k < n; k += 64) x[k] = vv[1 + k] / Tm;
                    wave_sync();
                    const unsigned long long s1 = prof ? wall_clock64() : 0ull;
                    const int pick = pick_action(x, n, e.greedy != 0, lane_uniform(e, i, st.ctr));
                    const unsigned long long s2 = prof ? wall_clock64() : 0ull;
                    lane_advance(e, i, st, pick, f.cand + ((size_t)i * f.cap + pick) * 8, vv[0], vv[1 + pick],
                                 n_full, l == 0);
                    if (prof) {
                        const unsigned long long s3 = wall_clock64();
                        tw[1] += s1 - s0;
                        tw[2] += s2 - s1;
                        tw[3] += s3 - s2;
                    }
                }
            }
            __syncthreads();
            tick(4);
            if (prof && t == 0) ph[5] += 1;
        }
        if (live && l == 0) lane_store(e, i, st);
    }
    if (prof) {
        unsigned long long* P = f.prof + (size_t)blockIdx.x * 16;
        if (t == 0)
            for (int k = 0; k < 6; ++k) atomicAdd(P + k, ph[k]);
        if (l == 0) {
            atomicAdd(P + 6, tj);
            for (int k = 0; k < 4; ++k) atomicAdd(P + 7 + k, tw[k]);
        }
    }
    if (t == 0) {
        atomicAdd(e.stats + 0, n_steps);
        atomicAdd(e.stats + 3, n_rows);
        atomicAdd(e.stats + 4, n_steps);
        atomicAdd(e.stats + 5, n_fb);
    }
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_fused(const bgx::FusedArgs* args, hipStream_t stream) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
        if (hipFuncSetAttribute((const void*)bgx::fused_step_kernel<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bgx::F_LDS) != hipSuccess ||
            hipFuncSetAttribute((const void*)bgx::fused_step_kernel<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bgx::F_LDS) != hipSuccess)
            return hipErrorInvalidValue;
    }
    if (args->n_steps <= 0 || args->e.L <= 0) return hipSuccess;
    if (args->cap < 1 || args->cap > bgx::F_OVL / 4 / bgx::FW) return hipErrorInvalidValue;
    // persistent: at most one workgroup per CU (LDS) and one tier-3 slice each
    const int groups = (args->e.L + bgx::FW - 1) / bgx::FW;
    int blocks = groups < n_cu ? groups : n_cu;
    if (blocks > args->ws_blocks) blocks = args->ws_blocks;
    if (args->prof)
        hipLaunchKernelGGL(bgx::fused_step_kernel<true>, dim3(blocks), dim3(64 * bgx::FW), bgx::F_LDS, stream, *args);
    else
        hipLaunchKernelGGL(bgx::fused_step_kernel<false>, dim3(blocks), dim3(64 * bgx::FW), bgx::F_LDS, stream, *args);
    return hipGetLastError();
}
