// bgx_encode.hip — K1: the 198-feature board encoder, plus board packing.
//
// Layout 0 (LIVE): ImmutableBoard.get_board_features (immutable_board.py:86-128)
//   f[96*pl + 4*i + c] = [n>=1, n>=2, n>=3, max(n-3,0)/2] for player pl, point i;
//   f[192..195] = bar1/2, off1/15, bar2/2, off2/15; f[196..197] = player flags.
// Layout 1 (interleaved, dead in the reference): generate_board_tensor.compute_features
//   (generate_board_tensor.py:98-140): per player 96 point features, bar/2, off/15.
// off/15 is produced as (float)(k / 15.0) — the value the reference stores
// (a Python double rounded into a float32 tensor).
//
// HBM-bound: 52 B in, 792 B out per board. Each thread writes one 16-byte
// float4 of the flat [n][198] output (fully coalesced dwordx4 stores); the
// board bytes it needs come through L1/L2.
#include "bgx_device.h"
#include "bgx_domain.h"
#include "bgx_kernels.h"

namespace bgx {

__constant__ float kOff15[16] = {
    (float)(0 / 15.0),  (float)(1 / 15.0),  (float)(2 / 15.0),  (float)(3 / 15.0),
    (float)(4 / 15.0),  (float)(5 / 15.0),  (float)(6 / 15.0),  (float)(7 / 15.0),
    (float)(8 / 15.0),  (float)(9 / 15.0),  (float)(10 / 15.0), (float)(11 / 15.0),
    (float)(12 / 15.0), (float)(13 / 15.0), (float)(14 / 15.0), (float)(15 / 15.0)};

BGX_DEV float feature(const uint8_t* b, int player, int layout, int f) {
    int pl, rest;
    if (f >= 196) return (f - 196) == player ? 1.0f : 0.0f;
    if (layout == 0) {
        if (f < 192) { pl = f / 96; rest = f - 96 * pl; }
        else {
            const int k = f - 192;   // bar1, off1, bar2, off2
            const int who = k >> 1;
            return (k & 1) ? kOff15[b[50 + who]] : (float)b[48 + who] * 0.5f;
        }
    } else {
        pl = f / 98;
        rest = f - 98 * pl;
        if (rest == 96) return (float)b[48 + pl] * 0.5f;
        if (rest == 97) return kOff15[b[50 + pl]];
    }
    const int n = b[24 * pl + (rest >> 2)];
    switch (rest & 3) {
        case 0: return n >= 1 ? 1.0f : 0.0f;
        case 1: return n >= 2 ? 1.0f : 0.0f;
        case 2: return n >= 3 ? 1.0f : 0.0f;
        default: return n > 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
}

__global__ __launch_bounds__(256) void encode_kernel(const uint8_t* __restrict__ boards,
                                                     const uint8_t* __restrict__ player, int n,
                                                     float* __restrict__ out, int layout) {
    const size_t total = (size_t)n * 198;
    const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
    for (size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < total; g += stride) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const size_t e = g + q;
            if (e < total) {
                const int row = (int)(e / 198);
                const int f = (int)(e - (size_t)row * 198);
                v[q] = feature(boards + (size_t)row * 52, player[row], layout, f);
            } else {
                v[q] = 0.0f;
            }
        }
        if (g + 4 <= total) {
            *(float4*)(out + g) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            for (int q = 0; q < 4 && g + q < total; ++q) out[g + q] = v[q];
        }
    }
}

// The engine's own packed boards (records, candidate rows) straight to
// features: one thread per (row, 4-feature quad), the row's two dwordx4 loads
// shared through L1 by the 50 quads of a row; the point count is the nibble of
// point i of player pl (word 3 pl + i / 8), bars / borne-off / the indicator
// come from word 6. Same values as encode_kernel on the unpacked board.
BGX_DEV float feature_packed(const uint32_t* w, int layout, int f) {
    const uint32_t s6 = w[6];
    const int player = (int)((s6 >> 16) & 1u);
    int pl, rest;
    if (f >= 196) return (f - 196) == player ? 1.0f : 0.0f;
    if (layout == 0) {
        if (f < 192) { pl = f / 96; rest = f - 96 * pl; }
        else {
            const int k = f - 192;   // bar1, off1, bar2, off2
            const int who = k >> 1;
            return (k & 1) ? kOff15[(s6 >> (8 + 4 * who)) & 15u] : (float)((s6 >> (4 * who)) & 15u) * 0.5f;
        }
    } else {
        pl = f / 98;
        rest = f - 98 * pl;
        if (rest == 96) return (float)((s6 >> (4 * pl)) & 15u) * 0.5f;
        if (rest == 97) return kOff15[(s6 >> (8 + 4 * pl)) & 15u];
    }
    const int i = rest >> 2;
    const int n = (int)((w[3 * pl + (i >> 3)] >> (4 * (i & 7))) & 15u);
    switch (rest & 3) {
        case 0: return n >= 1 ? 1.0f : 0.0f;
        case 1: return n >= 2 ? 1.0f : 0.0f;
        case 2: return n >= 3 ? 1.0f : 0.0f;
        default: return n > 3 ? (float)(n - 3) * 0.5f : 0.0f;
    }
}

__global__ __launch_bounds__(256) void encode_packed_kernel(const uint32_t* __restrict__ packed, int n,
                                                            float* __restrict__ out, int layout) {
    const size_t total = (size_t)n * 198;
    const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
    for (size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < total; g += stride) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const size_t e = g + q;
            if (e < total) {
                const int row = (int)(e / 198);
                const int f = (int)(e - (size_t)row * 198);
                const uint4* p = (const uint4*)(packed + (size_t)row * 8);
                const uint4 x = p[0], y = p[1];
                const uint32_t w[7] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z};
                v[q] = feature_packed(w, layout, f);
            } else {
                v[q] = 0.0f;
            }
        }
        if (g + 4 <= total) {
            *(float4*)(out + g) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            for (int q = 0; q < 4 && g + q < total; ++q) out[g + q] = v[q];
        }
    }
}

__global__ __launch_bounds__(256) void pack_kernel(const uint8_t* __restrict__ boards,
                                                   const uint8_t* __restrict__ player, int n,
                                                   uint32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* b = (const uint32_t*)(boards + (size_t)i * 52);
    uint32_t t[13], w[8];
#pragma unroll
    for (int k = 0; k < 13; ++k) t[k] = b[k];
    u8_to_packed(t, player ? (uint32_t)player[i] : 0u, w);
    uint4* o = (uint4*)(out + (size_t)i * 8);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ __launch_bounds__(256) void unpack_kernel(const uint32_t* __restrict__ packed, int n,
                                                     uint8_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* p = (const uint4*)(packed + (size_t)i * 8);
    const uint4 x = p[0], y = p[1];
    const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    uint32_t o[13];
    packed_to_u8(w, o);
    uint32_t* d = (uint32_t*)(out + (size_t)i * 52);
#pragma unroll
    for (int k = 0; k < 13; ++k) d[k] = o[k];
}

// Input-domain check of the stateless entry points (one thread per board;
// bgx_domain.h): flags[0] |= BGX_BADF_* bits, flags[1] = lowest offending
// index (atomicMin; the launcher presets ~0).
__global__ __launch_bounds__(256) void validate_kernel(const uint8_t* __restrict__ boards,
                                                       const uint8_t* __restrict__ player,
                                                       const uint8_t* __restrict__ dice, int n,
                                                       unsigned* __restrict__ flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned bad = domain_bits(boards + (size_t)i * 52, player ? (int)player[i] : -1,
                                     dice ? dice + 2 * (size_t)i : nullptr);
    if (bad) {
        atomicOr(&flags[0], bad);
        atomicMin(&flags[1], (unsigned)i);
    }
}

}  // namespace bgx

extern "C" hipError_t bgx_launch_validate(const uint8_t* boards, const uint8_t* player, const uint8_t* dice,
                                          int n, unsigned* flags, hipStream_t stream) {
    const unsigned init[2] = {0u, 0xFFFFFFFFu};
    hipError_t e = hipMemsetD32Async((hipDeviceptr_t)flags, init[0], 1, stream);
    if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)(flags + 1), init[1], 1, stream);
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(bgx::validate_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, boards, player, dice, n,
                       flags);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_encode(const uint8_t* boards, const uint8_t* player, int n,
                                        float* out, int layout, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const size_t quads = ((size_t)n * 198 + 3) / 4;
    size_t blocks = (quads + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(bgx::encode_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, boards, player,
                       n, out, layout);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_encode_packed(const uint32_t* packed, int n, float* out, int layout,
                                               hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const size_t quads = ((size_t)n * 198 + 3) / 4;
    size_t blocks = (quads + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(bgx::encode_packed_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, packed, n, out,
                       layout);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_pack(const uint8_t* boards, const uint8_t* player, int n,
                                      uint32_t* out, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::pack_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, boards, player, n,
                       out);
    return hipGetLastError();
}

extern "C" hipError_t bgx_launch_unpack(const uint32_t* packed, int n, uint8_t* out,
                                        hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(bgx::unpack_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, packed, n, out);
    return hipGetLastError();
}
