// bgx_mlp.hip — K3: fused encode + BackgammonPolicyNetwork forward on MFMA.
//
// Replaces ImmutableBoard.get_board_features (immutable_board.py:86-128) +
// BackgammonPolicyNetwork.forward (src/agents/policy_network.py:53-70) for a
// ragged batch of afterstates: V = w2 . sigmoid(W1 x + b1) + b2, W1 [128][198].
//
// Numerics ("split fp16"). Every live feature is exact in fp16
// once the two borne-off columns (193, 195) take the integer count k and W1's
// columns are pre-divided by 15; b1 rides in the K padding as column 198 with
// a constant feature. W1 is pre-multiplied by -log2(e) (so the accumulator is
// directly the exp2 argument of the sigmoid) and by one power of two 2^e
// (largest |w| in [2^14, 2^15), e capped at 13), the features by 2^-e (still
// exact: multiples of 0.5 * 2^-e, normal for e <= 13); residues below the fp16
// normal range carry absolute errors ~2^-25 / 2^e, negligible. W = W_hi + W_lo,
// both fp16; the MFMA multiplies are exact and accumulate in fp32, so two
// passes give ~fp32 accuracy (|dV| < 1e-5 on the trained checkpoint).
//
// Features for k-steps 0..11 come from a 256-entry LDS table: one byte of the
// packed board = the counts of two adjacent point slots -> their 8 fp16
// features (16 B, one ds_read_b128).
//
// MFMA: v_mfma_f32_32x32x16_f16 with A = W (32 hidden rows x 16 features) and
// B = X^T (16 features x 32 boards): the accumulator holds one board per lane
// column and 16 hidden rows per lane, so the value-head dot product is an
// in-register sum plus one cross-half shuffle. Features are built in
// registers from the 32-byte packed board (no feature tensor in HBM).
// W fragments (2 terms x 4 m-tiles x 13 k-steps x 64 lanes x 16 B = 104 KB)
// stay resident in LDS; one persistent 512-thread workgroup per CU.
#include "bgx_mlp.h"

#include <cstdlib>

namespace bgx {

BGX_DEV void load_rows(const MlpArgs& a, int n, int t, int NTq, int col, uint4& x, uint4& y) {
    const int row = t * 32 + col;
    x = make_uint4(0, 0, 0, 0);
    y = make_uint4(0, 0, 0, 0);
    (void)NTq;
    if (row < n) {
        const uint4* p = (const uint4*)(a.rows + (size_t)row * 8);
        x = p[0];
        y = p[1];
    }
}

// NT = board tiles of 32 per wave iteration (1: latency-bound small batches,
// 2: throughput; each A fragment read from LDS then feeds 2 MFMAs); NW =
// waves per block (one persistent block per CU). The next tile's rows and the
// next k-step's A / feature fragments are loaded while the current k-step's
// MFMAs run.
template <int NT, int NW>
__global__ __launch_bounds__(64 * NW) void mlp_kernel(MlpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    uint4* wf = lds;                                   // [NFRAG]
    uint4* lut = lds + NFRAG;                          // [256]
    float* w2s = (float*)(lds + NFRAG + 256);          // [128] value-head weights
    for (int i = threadIdx.x; i < NFRAG; i += blockDim.x) wf[i] = a.wfrag[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = lut_entry((uint32_t)i, a.feat_scale);
    for (int i = threadIdx.x; i < 128; i += blockDim.x) w2s[i] = a.rowc[i];

    int n = a.n_rows;
    if (a.n_rows_dev) n += (int)*a.n_rows_dev;
    if (a.n_max > 0 && n > a.n_max) n = a.n_max;
    const int tiles = (n + 32 * NT - 1) / (32 * NT);
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int nwaves = gridDim.x * NW;
    int t = blockIdx.x * NW + wave;
    uint4 px[NT], py[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) load_rows(a, n, t * NT + q, NT, col, px[q], py[q]);
    __syncthreads();
    for (; t < tiles; t += nwaves) {
        uint4 bx[NT], by[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            bx[q] = px[q];
            by[q] = py[q];
            load_rows(a, n, (t + nwaves) * NT + q, NT, col, px[q], py[q]);   // next tile
        }
        floatx16 acc[4][NT];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int q = 0; q < NT; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[m][q][r] = 0.0f;
        // fragment pipeline at (k-step, m-tile) granularity: the next (hi, lo)
        // A pair is read from LDS while the current pair's MFMAs run
        uint4 ch = wf[((0 * 4 + 0) * KSTEPS + 0) * 64 + lane];
        uint4 cl = wf[((1 * 4 + 0) * KSTEPS + 0) * 64 + lane];
        half8 b[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) b[q] = feat_frag(bx[q], by[q], 0, h, lut, a.feat_scale);
#pragma unroll 1
        for (int s = 0; s < KSTEPS; ++s) {
            const int sn = s + 1 < KSTEPS ? s + 1 : s;
            half8 nb[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) nb[q] = feat_frag(bx[q], by[q], sn, h, lut, a.feat_scale);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int s2 = m < 3 ? s : sn, m2 = m < 3 ? m + 1 : 0;
                const uint4 nh = wf[((0 * 4 + m2) * KSTEPS + s2) * 64 + lane];
                const uint4 nl = wf[((1 * 4 + m2) * KSTEPS + s2) * 64 + lane];
#pragma unroll
                for (int q = 0; q < NT; ++q) {
                    acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ch, b[q], acc[m][q], 0, 0, 0);
                    acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&cl, b[q], acc[m][q], 0, 0, 0);
                }
                ch = nh;
                cl = nl;
            }
#pragma unroll
            for (int q = 0; q < NT; ++q) b[q] = nb[q];
        }
        if (a.zout) {
            // the 2-ply root launch: the rows' accumulators for the reply launch's
            // evaluation by difference (mlp_kernel_delta), 64 contiguous floats per lane
#pragma unroll
            for (int q = 0; q < NT; ++q) {
                const int row = (t * NT + q) * 32 + col;
                if (row >= a.z_base && row < n) {
                    v4f* zp = (v4f*)(a.zout + (size_t)(row - a.z_base) * 128 + 64 * h);
#pragma unroll
                    for (int m = 0; m < 4; ++m)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const v4f zv = {acc[m][q][4 * i], acc[m][q][4 * i + 1], acc[m][q][4 * i + 2],
                                            acc[m][q][4 * i + 3]};
                            zp[4 * m + i] = zv;
                        }
                }
            }
        }
        float v[NT];
        // sigmoid(h) = 1 / (1 + 2^acc) (acc = -h log2 e); w2 of the lane's hidden
        // rows j0 = 32m + (r & 3) + 8(r >> 2) + 4h from LDS, four at a time;
        // summed in the canonical order (bgx_mlp.h, epilogue order)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float pm[NT];
#pragma unroll
            for (int q = 0; q < NT; ++q) pm[q] = 0.0f;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 c4 = *(const float4*)(w2s + 32 * m + 8 * g + 4 * h);
                const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int r = 4 * g + k;
#pragma unroll
                    for (int q = 0; q < NT; ++q) {
                        const float ex = __builtin_amdgcn_exp2f(acc[m][q][r]);
                        pm[q] = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), pm[q]);
                    }
                    if ((r & 1) == 1) __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int q = 0; q < NT; ++q) v[q] = m == 0 ? pm[q] : v[q] + pm[q];
        }
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            v[q] += __shfl_xor(v[q], 32, 64);
            const int row = (t * NT + q) * 32 + col;
            if (h == 0 && row < n) a.out[row] = v[q] + a.b2;
        }
    }
}

// Throughput kernel (2 tiles of 32 boards per wave, 8 waves, one workgroup per
// CU): all 13 feature fragments of a tile pair are built once (104 VGPRs),
// then the four 32-row hidden tiles m run one after another into two
// alternating accumulator sets; the sigmoid + w2 dot product of tile m-1 runs
// beside tile m's 52 MFMAs (the VALU / transcendental issue fits in the MFMA
// gaps). The last m-tile's epilogue is carried into the next tile pair's
// first m-tile (acc[1] stays live across the iteration), so only each wave's
// last epilogue is exposed. Each wave's next tile pair of rows is staged
// global -> LDS by two global_load_lds_dwordx4 (no VGPRs: the kernel is at its
// register cap) while the current pair's 208 MFMAs run. Same accumulation and
// epilogue order as every MLP kernel (bgx_mlp.h).
// (Measured and rejected, DESIGN.md §4: skipping all-zero k-steps -- the
// branches break the MFMA / epilogue interleave -- and a 12-wave variant that
// rebuilds the feature fragments per m-tile.)
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) void* glb_vp;

// epi_pair with the w2 base (w2s + 4 h) as an LDS pointer: the reads take
// constant offsets from one register
BGX_DEV void epi_pair_l(const floatx16& acc, int m, int r0, lds_fp w2h, float& v) {
    const v2f c = *(__attribute__((address_space(3))) const v2f*)(w2h + 32 * m + (r0 & 3) + 8 * (r0 >> 2));
    const float e0 = __builtin_amdgcn_exp2f(acc[r0]), e1 = __builtin_amdgcn_exp2f(acc[r0 + 1]);
    v = fmaf(c.x, __builtin_amdgcn_rcpf(1.0f + e0), v);
    v = fmaf(c.y, __builtin_amdgcn_rcpf(1.0f + e1), v);
}
constexpr int IL_NW = 8;
constexpr int IL_RB = 128;   // uint4 per staged tile pair (64 rows x 32 B)

// rows 64 t .. 64 t + 63 -> dst[2 r], dst[2 r + 1] (wave-uniform LDS base +
// 16 B per lane); rows past the buffer's capacity read its last row (their
// V is never stored)
BGX_DEV void il_stage(const uint32_t* rows, int t, int cap, uint4* dst) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int row = 64 * t + 32 * i + (lane >> 1);
        row = row < cap ? row : cap - 1;
        const uint4* src = (const uint4*)(rows + (size_t)row * 8) + (lane & 1);
        __builtin_amdgcn_global_load_lds((glb_vp)(void*)src, (lds_vp)(void*)(dst + 64 * i), 16, 0, 0);
    }
}

__global__ __launch_bounds__(64 * IL_NW) void mlp_kernel_il(MlpArgs a) {
    constexpr int NT = 2;
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    uint4* wf = lds;                                   // [NFRAG]
    uint4* lut = lds + NFRAG;                          // [256]
    float* w2s = (float*)(lds + NFRAG + 256);          // [128] value-head weights
    uint4* rbuf = lds + NFRAG + 256 + 32;              // [IL_NW][2][IL_RB] staged rows
    int n = a.n_rows;
    if (a.n_rows_dev) n += (int)*a.n_rows_dev;
    if (a.n_max > 0 && n > a.n_max) n = a.n_max;
    const int cap = a.n_max > 0 ? a.n_max : n;
    const int tiles = (n + 32 * NT - 1) / (32 * NT);
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int nwaves = gridDim.x * IL_NW;
    uint4* rb = rbuf + wave * 2 * IL_RB;
    // fragment bases: hi terms wf[0 .. 52*64), lo terms from wf + 52*64; each
    // read then fits a ds_read offset (< 64 KB). The asm (per tile pair) hides
    // the bases' relation and their loop invariance, so the compiler neither
    // folds them into one base plus per-fragment address registers nor hoists
    // the fragment reads out of the loop (into spills).
    lds_u4p wfh = (lds_u4p)(wf + lane);
    lds_u4p wfl = (lds_u4p)(wf + 4 * KSTEPS * 64 + lane);
    lds_fp w2h = (lds_fp)(w2s + 4 * h);
    int t = blockIdx.x * IL_NW + wave;
    if (t < tiles) il_stage(a.rows, t, cap, rb);
    for (int i = threadIdx.x; i < NFRAG; i += blockDim.x) wf[i] = a.wfrag[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = lut_entry((uint32_t)i, a.feat_scale);
    for (int i = threadIdx.x; i < 128; i += blockDim.x) w2s[i] = a.rowc[i];
    __syncthreads();
    float v[NT] = {0.0f, 0.0f}, pm[NT] = {0.0f, 0.0f};   // canonical epilogue order (bgx_mlp.h)
    floatx16 acc[2][NT];
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[1][q][r] = 0.0f;
    int tp = -1;   // tile pair whose m-tile 3 accumulators are in acc[1]
    for (int it = 0; t < tiles; t += nwaves, ++it) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this pair's staged rows landed
        const uint4* cb = rb + (it & 1) * IL_RB;
        half8 b[KSTEPS][NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            const uint4 bx = cb[2 * (32 * q + col)], by = cb[2 * (32 * q + col) + 1];
#pragma unroll
            for (int s = 0; s < KSTEPS - 1; ++s) b[s][q] = feat_frag(bx, by, s, h, lut, a.feat_scale);
            b[KSTEPS - 1][q] = feat_frag(make_uint4(0, 0, 0, 0), make_uint4(0, 0, by.z, 0), KSTEPS - 1, h, lut,
                                         a.feat_scale);
        }
        if (t + nwaves < tiles) il_stage(a.rows, t + nwaves, cap, rb + ((it + 1) & 1) * IL_RB);
        asm volatile("" : "+v"(wfh));
        asm volatile("" : "+v"(wfl));
        asm volatile("" : "+v"(w2h));
        v4u ah = wfh[0];
        v4u al = wfl[0];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int cur = m & 1, prv = cur ^ 1;
            const int mp = m > 0 ? m - 1 : 3;   // m-tile whose epilogue runs beside these MFMAs
#pragma unroll
            for (int q = 0; q < NT; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[cur][q][r] = 0.0f;
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                const int mn = s + 1 < KSTEPS ? m : (m + 1 < 4 ? m + 1 : m);
                const int sn = s + 1 < KSTEPS ? s + 1 : 0;
                const v4u nh = wfh[(mn * KSTEPS + sn) * 64];
                const v4u nl = wfl[(mn * KSTEPS + sn) * 64];
#pragma unroll
                for (int q = 0; q < NT; ++q) {
                    acc[cur][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ah), b[s][q], acc[cur][q], 0, 0, 0);
                    acc[cur][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, al), b[s][q], acc[cur][q], 0, 0, 0);
                }
                // m-tile mp's epilogue spread over the 13 k-steps: its 16 row pairs
                // (p: tile p & 1, rows 2 (p >> 1), +1; ascending per tile), two
                // per step in steps 0..2, one per step after
                const int p_lo = s < 3 ? 2 * s : s + 3;
                const int p_n = s < 3 ? 2 : 1;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    if (k >= p_n) break;
                    const int p = p_lo + k;
                    epi_pair_l(acc[prv][p & 1], mp, 2 * (p >> 1), w2h, pm[p & 1]);
                }
                if (s == KSTEPS - 1) {
                    if (m == 0) {
                        // the previous tile pair is complete: V = (v_0 + v_1) + b2
#pragma unroll
                        for (int q = 0; q < NT; ++q) {
                            float vv = v[q] + pm[q];
                            vv += __shfl_xor(vv, 32, 64);
                            const int row = (tp * NT + q) * 32 + col;
                            if (tp >= 0 && h == 0 && row < n) a.out[row] = vv + a.b2;
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < NT; ++q) v[q] = m == 1 ? pm[q] : v[q] + pm[q];
                    }
#pragma unroll
                    for (int q = 0; q < NT; ++q) pm[q] = 0.0f;
                }
                ah = nh;
                al = nl;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        tp = t;
    }
    if (tp >= 0) {
#pragma unroll
        for (int r = 0; r < 16; r += 2)
#pragma unroll
            for (int q = 0; q < NT; ++q) epi_pair_l(acc[1][q], 3, r, w2h, pm[q]);
#pragma unroll
        for (int q = 0; q < NT; ++q) {
            float vv = v[q] + pm[q];
            vv += __shfl_xor(vv, 32, 64);
            const int row = (tp * NT + q) * 32 + col;
            if (h == 0 && row < n) a.out[row] = vv + a.b2;
        }
    }
}

// ---------------------------------------------------------------------------
// The 2-ply reply values by difference from the root (round 6). A reply
// board is its root (the candidate it answers, two_ply.py:93-150) after the
// opponent's move: it differs from the root only at the points the move
// touched, the bars / borne-off counts and the side to move. The root launch
// (mlp_kernel with zout) writes each candidate's hidden-layer accumulators,
// so a reply's accumulator is root + W . (x_reply - x_root), and only the
// k-steps where some row of the 32-row tile differs from its root contribute:
// k-step s < 12 covers bytes 2 s and 2 s + 1 of the packed board (four point
// slots of one player), k-step 12 the bars, borne-off counts and side to move
// (always run). In self-play ~7.7 of the 13 k-steps run per tile (replies to
// one root touch ~12 of the 24 point-pair bytes; tools/probe/delta_ksteps.py).
// The pairing of bytes into k-steps is the fixed one, so a row's value does not
// depend on the rows it shares a tile with (a k-step where its own difference
// is zero adds exact zeros): the same bits whichever tile, wave or run.
// Feature differences are exact in fp16 (multiples of 0.5 * 2^-e within
// +-15 * 2^-e), the MFMA products exact, the sums fp32: V within ~1e-6 of the
// full evaluation (tests/test_cpuwave.py on the shipped checkpoint), so the
// north_star tolerance 1e-5 holds (test_gpu_scale.py per-candidate W at the
// bench shape, test_gpu_replay.py golden W). One 32-row tile per wave
// iteration, 8 waves per CU, the next tile's rows staged by LDS-DMA, the next
// k-step's A fragments read ahead of the current MFMAs; the epilogue (root
// accumulator added, sigmoid, value head) in the canonical order.
constexpr int DL_NW = 8;
constexpr int DL_RB = 64;   // uint4 per staged tile (32 rows x 32 B)

// rows 32 t .. 32 t + 31 -> dst (16 B per lane); rows past the buffer's
// capacity read its last row (their V is never stored)
BGX_DEV void dl_stage(const uint32_t* rows, int t, int cap, uint4* dst) {
    const int lane = (int)(threadIdx.x & 63);
    int row = 32 * t + (lane >> 1);
    row = row < cap ? row : cap - 1;
    const uint4* src = (const uint4*)(rows + (size_t)row * 8) + (lane & 1);
    __builtin_amdgcn_global_load_lds((glb_vp)(void*)src, (lds_vp)(void*)dst, 16, 0, 0);
}

// Per wave iteration (tile t): t's root boards and root accumulators are
// requested, the previous tile's epilogue runs (covering the boards'
// latency), then t's k-step mask (ballots), its MFMAs (covering the root
// accumulators'), and the root accumulators are added; the next k-step's A
// fragments and LUT entries are read ahead of the current MFMAs.
__global__ __launch_bounds__(64 * DL_NW) void mlp_kernel_delta(MlpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    uint4* wf = lds;                                   // [NFRAG]
    uint4* lut = lds + NFRAG;                          // [256]
    float* w2s = (float*)(lds + NFRAG + 256);          // [128] value-head weights
    uint4* rbuf = lds + NFRAG + 256 + 32;              // [DL_NW][2][DL_RB] staged rows
    int n = a.n_rows;
    if (a.n_rows_dev) n += (int)*a.n_rows_dev;
    if (a.n_max > 0 && n > a.n_max) n = a.n_max;
    const int cap = a.n_max > 0 ? a.n_max : n;
    const int tiles = (n + 31) / 32;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int nwaves = gridDim.x * DL_NW;
    uint4* rb = rbuf + wave * 2 * DL_RB;
    int t = blockIdx.x * DL_NW + wave;
    if (t < tiles) dl_stage(a.rows, t, cap, rb);
    for (int i = threadIdx.x; i < NFRAG; i += blockDim.x) wf[i] = a.wfrag[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = lut_entry((uint32_t)i, a.feat_scale);
    for (int i = threadIdx.x; i < 128; i += blockDim.x) w2s[i] = a.rowc[i];
    __syncthreads();
    // fragment bases (hi terms, lo terms; each m-tile's fragments at a constant
    // offset below 64 KB from its base)
    const lds_u4p wfh = (lds_u4p)(wf + lane);
    const lds_u4p wfl = (lds_u4p)(wf + 4 * KSTEPS * 64 + lane);
    const lds_fp w2h = (lds_fp)(w2s + 4 * h);
    floatx16 acc[4];
    v4f z[16];
    int tp = -1;   // tile whose accumulators (acc) and root accumulators (z) await the epilogue
    // sigmoid and the value head in the canonical order (bgx_mlp.h) over the
    // tile's complete accumulators (root + difference)
    auto epilogue = [&](int tt) {
        float v = 0.0f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float pm = 0.0f;
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const v4f c4 = *(__attribute__((address_space(3))) const v4f*)(w2h + 32 * m + 8 * gq);
                const float cy[4] = {c4[0], c4[1], c4[2], c4[3]};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float ex = __builtin_amdgcn_exp2f(acc[m][4 * gq + k]);
                    pm = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), pm);
                }
            }
            v = m == 0 ? pm : v + pm;
        }
        v += __shfl_xor(v, 32, 64);
        const int row = tt * 32 + col;
        if (h == 0 && row < n) a.out[row] = v + a.b2;
    };
    for (int it = 0; t < tiles; t += nwaves, ++it) {
        // this tile's staged rows (and tp's z) landed: vmcnt(0) as the builtin
        // (0xF70: expcnt and lgkmcnt at their maxima), which the compiler's wait
        // insertion sees, so it does not also wait before the k-loop's LDS reads
        __builtin_amdgcn_s_waitcnt(0xF70);
        wave_sync();   // (host emulation: every lane's staging copy is done)
        const uint4* cb = rb + (it & 1) * DL_RB;
        const uint4 bx = cb[2 * col], by = cb[2 * col + 1];
        const int row = t * 32 + col;
        // the row's root (word 7 = root slot; stale rows past the records: clamped)
        const uint32_t slot = by.w < (uint32_t)a.n_slots ? by.w : (uint32_t)(a.n_slots - 1);
        int rr = a.root_sel ? a.root_sel[slot] : a.root_base + (int)slot;
        rr = rr < a.root_base ? a.root_base : (rr >= a.root_base + a.n_roots ? a.root_base + a.n_roots - 1 : rr);
        const uint4* rp = (const uint4*)(a.root_rows + (size_t)rr * 8);
        const uint4 rx = rp[0], ry = rp[1];
        // the root accumulators, added to this tile's after its MFMAs (~2 epilogue
        // and MFMA phases from now)
        const v4f* zp = (const v4f*)(a.zt + (size_t)(rr - a.root_base) * 128 + 64 * h);
#pragma unroll
        for (int i = 0; i < 16; ++i) z[i] = zp[i];
        if (tp >= 0) epilogue(tp);   // the previous tile, while the root boards arrive
        // the tile's k-steps: k-step s < 12 covers bytes 2 s, 2 s + 1 of the
        // packed board (its two lane halves), so it runs iff some row of the tile
        // differs from its root there; k-step 12 (bars, borne-off, side to move)
        // always runs (the side to move differs between a root and its replies).
        // A row's result does not depend on the tile it shares: a k-step where
        // its own difference is zero adds exact zeros, and the pairing of bytes
        // into k-steps is the fixed one (a pairing by the tile's changes made V
        // depend on which rows share a tile: ~1e-8, run to run)
        uint32_t mrem = 1u << 12;
        {
            const bool live = row < n;
            const uint32_t d[6] = {bx.x ^ rx.x, bx.y ^ rx.y, bx.z ^ rx.z, bx.w ^ rx.w, by.x ^ ry.x, by.y ^ ry.y};
#pragma unroll
            for (int s2 = 0; s2 < 12; ++s2)
                mrem |= ballot(live && ((d[s2 >> 1] >> (16 * (s2 & 1))) & 0xFFFFu) != 0u) ? 1u << s2 : 0u;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] = 0.0f;
        // k-step s's feature difference: the two LUT entries (k-step 12: the bars,
        // borne-off counts and side to move, dmisc; the bias cancels). The LUT
        // reads of the next k-step are issued before its A fragment reads and
        // subtracted one iteration later, so waiting for them never waits for
        // the fragments (LDS reads complete in order)
        half8 dmisc;
        {
            const half8 f1 = feat_frag(make_uint4(0, 0, 0, 0), make_uint4(0, 0, by.z, 0), KSTEPS - 1, h, lut,
                                       a.feat_scale);
            const half8 f0 = feat_frag(make_uint4(0, 0, 0, 0), make_uint4(0, 0, ry.z, 0), KSTEPS - 1, h, lut,
                                       a.feat_scale);
            dmisc = f1 - f0;
        }
        // (selects on the bits of the uniform k-step index: a chain of equality
        // tests on it became a private array in scratch)
        auto lut_byte = [&](const uint4& x, const uint4& y, int s2) -> uint32_t {
            const int s3 = s2 < 12 ? s2 : 0;
            const bool odd = (s3 & 2) != 0;
            const uint32_t w01 = odd ? x.y : x.x, w23 = odd ? x.w : x.z, w45 = odd ? y.y : y.x;
            const uint32_t word = s3 < 4 ? w01 : (s3 < 8 ? w23 : w45);
            return (word >> (8 * (2 * (s3 & 1) + h))) & 0xFFu;
        };
        // two fragment sets in turn (ping-pong): k-step i's MFMAs use set i & 1,
        // read during k-step i - 1; the reads of k-step i + 1 into the other set
        // are issued ahead of k-step i's MFMAs (no register copies between sets)
        uint4 fr[2], fq[2];
        v4u ah[2][4], al[2][4];
        int ks[2];
        auto issue = [&](int q) {   // the next k-step's LUT entries, then its A fragments, into set q
            const int s2 = __ffs(mrem) - 1;
            mrem &= mrem - 1u;
            ks[q] = s2;
            fr[q] = lut[lut_byte(bx, by, s2)];
            fq[q] = lut[lut_byte(rx, ry, s2)];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                ah[q][m] = wfh[(m * KSTEPS + s2) * 64];
                al[q][m] = wfl[(m * KSTEPS + s2) * 64];
            }
        };
        auto phase = [&](int q) {
            const half8 bd = *(const half8*)&fr[q] - *(const half8*)&fq[q];
            const half8 b = ks[q] < 12 ? bd : dmisc;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ah[q][m]), b, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, al[q][m]), b, acc[m], 0, 0, 0);
            }
        };
        issue(0);
        for (;;) {
            const bool more0 = mrem != 0u;
            if (more0) issue(1);
            phase(0);
            if (!more0) break;
            const bool more1 = mrem != 0u;
            if (more1) issue(0);
            phase(1);
            if (!more1) break;
        }
        // accumulator = difference + root (the fp32 sums of the root launch)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] += z[4 * m + (r >> 2)][r & 3];
        // the next tile's rows, staged after the MFMAs: an LDS-DMA in flight makes
        // the compiler wait for every vector-memory operation (the root
        // accumulators too) before each LDS read
        if (t + nwaves < tiles) dl_stage(a.rows, t + nwaves, cap, rb + ((it + 1) & 1) * DL_RB);
        tp = t;
    }
    if (tp >= 0) epilogue(tp);
}

// Generic fp32-input value (bgx_value: arbitrary x, plain fp32 FMA) — parity
// entry point, not the hot path. One 128-thread block per 8 rows.
__global__ __launch_bounds__(128) void value_f32_kernel(const float* __restrict__ x, int n,
                                                        const float* __restrict__ W1,
                                                        const float* __restrict__ b1,
                                                        const float* __restrict__ w2, float b2,
                                                        float* __restrict__ out) {
    __shared__ float xs[8][198];
    __shared__ float red[8][128];
    const int r0 = blockIdx.x * 8;
    for (int i = threadIdx.x; i < 8 * 198; i += 128) {
        const int r = i / 198, k = i - 198 * r;
        xs[r][k] = (r0 + r < n) ? x[(size_t)(r0 + r) * 198 + k] : 0.0f;
    }
    __syncthreads();
    const int j = threadIdx.x;
    float acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = 0.0f;
    for (int k = 0; k < 198; ++k) {
        const float wv = W1[(size_t)j * 198 + k];
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = fmaf(wv, xs[r][k], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) red[r][j] = w2[j] / (1.0f + expf(-(acc[r] + b1[j])));
    __syncthreads();
    for (int s = 64; s >= 1; s >>= 1) {
        if (j < s)
#pragma unroll
            for (int r = 0; r < 8; ++r) red[r][j] += red[r][j + s];
        __syncthreads();
    }
    if (j < 8 && r0 + j < n) out[r0 + j] = red[j][0] + b2;
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_mlp(const bgx::MlpArgs* args, hipStream_t stream) {
    // per device (one process may drive several GPUs: multi/worker.py gives
    // worker 0 GPUs 0 and 7): the CU count and the kernels' dynamic-LDS opt-in
    static int n_cu_dev[64] = {0};
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur < 0 || cur >= 64) cur = 0;
    int& n_cu = n_cu_dev[cur];
    const int lds = bgx::NFRAG * 16 + 256 * 16 + 128 * 4;
    const int lds_il = lds + bgx::IL_NW * 2 * bgx::IL_RB * 16;
    const int lds_dl = lds + bgx::DL_NW * 2 * bgx::DL_RB * 16;
    if (!n_cu) {
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, cur) != hipSuccess || n_cu <= 0)
            n_cu = 256;
        if (hipFuncSetAttribute((const void*)bgx::mlp_kernel<1, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lds) != hipSuccess ||
            hipFuncSetAttribute((const void*)bgx::mlp_kernel_il, hipFuncAttributeMaxDynamicSharedMemorySize, lds_il) !=
                hipSuccess ||
            hipFuncSetAttribute((const void*)bgx::mlp_kernel_delta, hipFuncAttributeMaxDynamicSharedMemorySize, lds_dl) !=
                hipSuccess)
            return hipErrorInvalidValue;
    }
    if (args->zt) {   // the 2-ply replies by difference from their roots (8 waves, one tile each)
        int blocks = n_cu;
        if (!args->n_rows_dev) {
            const int need = ((args->n_rows + 31) / 32 + bgx::DL_NW - 1) / bgx::DL_NW;
            if (need < blocks) blocks = need;
            if (blocks <= 0) return hipSuccess;
        }
        if (args->n_slots <= 0 || args->n_roots <= 0 || !args->root_rows) return hipErrorInvalidValue;
        hipLaunchKernelGGL(bgx::mlp_kernel_delta, dim3(blocks), dim3(64 * bgx::DL_NW), lds_dl, stream, *args);
        return hipGetLastError();
    }
    // nt = 1: latency-bound small batches (one 32-board tile per wave, 16-wave
    // blocks); nt = 2: throughput (the interleaved-epilogue kernel, 8 waves)
    const int nt = args->nt == 2 ? 2 : 1;
    const int nw = nt == 2 ? 8 : 16;
    int blocks = n_cu;
    if (!args->n_rows_dev) {
        const int tiles = (args->n_rows + 32 * nt - 1) / (32 * nt);
        const int need = (tiles + nw - 1) / nw;
        if (need < blocks) blocks = need;
        if (blocks <= 0) return hipSuccess;
    }
    if (nt == 2)
        hipLaunchKernelGGL(bgx::mlp_kernel_il, dim3(blocks), dim3(64 * bgx::IL_NW), lds_il, stream, *args);
    else
        hipLaunchKernelGGL((bgx::mlp_kernel<1, 16>), dim3(blocks), dim3(1024), lds, stream, *args);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_value_f32(const float* x, int n, const float* W1, const float* b1,
                                           const float* w2, float b2, float* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::value_f32_kernel, dim3((n + 7) / 8), dim3(128), 0, stream, x, n, W1, b1,
                       w2, b2, out);
    return hipGetLastError();
}
