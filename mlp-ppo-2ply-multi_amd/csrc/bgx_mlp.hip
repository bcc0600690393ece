// bgx_mlp.hip — K3: fused encode + BackgammonPolicyNetwork forward on MFMA.
//
// Replaces ImmutableBoard.get_board_features (immutable_board.py:86-128) +
// BackgammonPolicyNetwork.forward (src/agents/policy_network.py:53-70) for a
// ragged batch of afterstates: V = w2 . sigmoid(W1 x + b1) + b2, W1 [128][198].
//
// Numerics ("split fp16"). Every live feature is exact in fp16
// once the two borne-off columns (193, 195) take the integer count k and W1's
// columns are pre-divided by 15. Each hidden row j is scaled by 2^e_j (so its
// largest |w| sits in [2^14, 2^15): no fp16 overflow, no subnormal residue)
// and split W = W_hi + W_lo, both fp16; the MFMA multiplies are exact and
// accumulate in fp32, so two passes give ~fp32 accuracy (|dV| << 1e-5).
//
// MFMA: v_mfma_f32_32x32x16_f16 with A = W (32 hidden rows x 16 features) and
// B = X^T (16 features x 32 boards): the accumulator holds one board per lane
// column and 16 hidden rows per lane, so the value-head dot product is an
// in-register sum plus one cross-half shuffle. Features are built in
// registers from the 32-byte packed board (no feature tensor in HBM).
// W fragments (2 terms x 4 m-tiles x 13 k-steps x 64 lanes x 16 B = 104 KB)
// stay resident in LDS; one persistent 512-thread workgroup per CU.
#include "bgx_device.h"
#include "bgx_kernels.h"

namespace bgx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KSTEPS = 13;   // 208 = 13 x 16 >= 198
constexpr int NFRAG = 2 * 4 * KSTEPS * 64;

BGX_DEV _Float16 hf(float v) { return (_Float16)v; }

// B fragment (8 features of one board) for k-step s (0..12), lane half h
BGX_DEV half8 feat_frag(const uint4 x, const uint4 y, int s, int h) {
    half8 f;
    if (s < 12) {
        // point slots q0 = 4s + 2h and q0 + 1: word s >> 1, nibbles 4(s&1) + 2h (+1)
        const int wi = s >> 1;
        uint32_t word = x.x;
        word = wi == 1 ? x.y : word;
        word = wi == 2 ? x.z : word;
        word = wi == 3 ? x.w : word;
        word = wi == 4 ? y.x : word;
        word = wi == 5 ? y.y : word;
        const int nb = 4 * (s & 1) + 2 * h;
        const uint32_t two = word >> (4 * nb);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = (int)((two >> (4 * t)) & 15u);
            f[4 * t + 0] = n >= 1 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * t + 1] = n >= 2 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * t + 2] = n >= 3 ? (_Float16)1.0f : (_Float16)0.0f;
            f[4 * t + 3] = (_Float16)(n > 3 ? (float)(n - 3) * 0.5f : 0.0f);
        }
    } else {
        const uint32_t s6 = y.z;
        const float on = h == 0 ? 1.0f : 0.0f;
        const uint32_t flag = (s6 >> 16) & 1u;
        f[0] = hf(on * (float)(s6 & 15u) * 0.5f);          // bar1 / 2
        f[1] = hf(on * (float)((s6 >> 8) & 15u));          // off1 (W col / 15)
        f[2] = hf(on * (float)((s6 >> 4) & 15u) * 0.5f);   // bar2 / 2
        f[3] = hf(on * (float)((s6 >> 12) & 15u));         // off2 (W col / 15)
        f[4] = hf(on * (flag == 0u ? 1.0f : 0.0f));        // PLAYER1 to play
        f[5] = hf(on * (flag == 1u ? 1.0f : 0.0f));        // PLAYER2 to play
        f[6] = (_Float16)0.0f;
        f[7] = (_Float16)0.0f;
    }
    return f;
}

__global__ __launch_bounds__(512) void mlp_kernel(MlpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds[];
    uint4* wf = lds;                                   // [NFRAG]
    float4* rc = (float4*)(lds + NFRAG);               // [128]
    for (int i = threadIdx.x; i < NFRAG; i += blockDim.x) wf[i] = a.wfrag[i];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) rc[i] = ((const float4*)a.rowc)[i];
    __syncthreads();

    int n = a.n_rows;
    if (a.n_rows_dev) n += (int)*a.n_rows_dev;
    if (a.n_max > 0 && n > a.n_max) n = a.n_max;
    const int tiles = (n + 31) >> 5;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int col = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int waves = blockDim.x >> 6;
    for (int t = blockIdx.x * waves + wave; t < tiles; t += gridDim.x * waves) {
        const int row = t * 32 + col;
        uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
        if (row < n) {
            const uint4* p = (const uint4*)(a.rows + (size_t)row * 8);
            x = p[0];
            y = p[1];
        }
        floatx16 acc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] = 0.0f;
#pragma unroll 1
        for (int s = 0; s < KSTEPS; ++s) {
            const half8 b = feat_frag(x, y, s, h);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint4 ah = wf[((0 * 4 + m) * KSTEPS + s) * 64 + lane];
                const uint4 al = wf[((1 * 4 + m) * KSTEPS + s) * 64 + lane];
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ah, b, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&al, b, acc[m], 0, 0, 0);
            }
        }
        float v = 0.0f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int j = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float4 c = rc[j];
                const float hv = fmaf(acc[m][r], c.x, c.z);
                v = fmaf(c.y, 1.0f / (1.0f + __expf(-hv)), v);
                if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
        v += __shfl_xor(v, 32, 64);
        if (h == 0 && row < n) a.out[row] = v + a.b2;
    }
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
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
        if (n_cu <= 0) n_cu = 256;
        hipFuncSetAttribute((const void*)bgx::mlp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            bgx::NFRAG * 16 + 128 * 16);
    }
    int blocks = n_cu;
    if (!args->n_rows_dev) {
        const int tiles = (args->n_rows + 31) / 32;
        const int need = (tiles + 7) / 8;
        if (need < blocks) blocks = need;
        if (blocks <= 0) return hipSuccess;
    }
    hipLaunchKernelGGL(bgx::mlp_kernel, dim3(blocks), dim3(512), bgx::NFRAG * 16 + 128 * 16, stream,
                       *args);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_value_f32(const float* x, int n, const float* W1, const float* b1,
                                           const float* w2, float b2, float* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::value_f32_kernel, dim3((n + 7) / 8), dim3(128), 0, stream, x, n, W1, b1,
                       w2, b2, out);
    return hipGetLastError();
}
