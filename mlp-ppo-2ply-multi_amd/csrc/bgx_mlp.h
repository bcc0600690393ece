// bgx_mlp.h — K3 device code (split-fp16 fragments, fused feature build), shared by
// the MLP kernels (bgx_mlp.hip) and the fused 1-ply lane kernel (bgx_fused.hip).
// Numerics and layout: see the header comment of bgx_mlp.hip.
#pragma once
#include "bgx_device.h"
#include "bgx_kernels.h"

namespace bgx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KSTEPS = 13;   // 208 = 13 x 16 >= 198
constexpr int NFRAG = 2 * 4 * KSTEPS * 64;

BGX_DEV _Float16 hf(float v) { return (_Float16)v; }

// B fragment (8 features of one board) for k-step s (0..12), lane half h
BGX_DEV half8 feat_frag(const uint4 x, const uint4 y, int s, int h, const uint4* lut, float sc) {
    if (s < 12) {
        // point slots q0 = 4s + 2h and q0 + 1 = byte (2(s&1) + h) of word s >> 1
        const int wi = s >> 1;
        uint32_t word = x.x;
        word = wi == 1 ? x.y : word;
        word = wi == 2 ? x.z : word;
        word = wi == 3 ? x.w : word;
        word = wi == 4 ? y.x : word;
        word = wi == 5 ? y.y : word;
        const uint32_t byte = (word >> (8 * (2 * (s & 1) + h))) & 0xFFu;
        const uint4 f = lut[byte];
        return *(const half8*)&f;
    }
    half8 f;
    const uint32_t s6 = y.z;
    const float on = h == 0 ? sc : 0.0f;   // features carry the 2^-e scale
    const uint32_t flag = (s6 >> 16) & 1u;
    f[0] = hf(on * (float)(s6 & 15u) * 0.5f);          // bar1 / 2
    f[1] = hf(on * (float)((s6 >> 8) & 15u));          // off1 (W col / 15)
    f[2] = hf(on * (float)((s6 >> 4) & 15u) * 0.5f);   // bar2 / 2
    f[3] = hf(on * (float)((s6 >> 12) & 15u));         // off2 (W col / 15)
    f[4] = hf(on * (flag == 0u ? 1.0f : 0.0f));        // PLAYER1 to play
    f[5] = hf(on * (flag == 1u ? 1.0f : 0.0f));        // PLAYER2 to play
    f[6] = hf(on);                                     // bias feature (W col 198 = b1)
    f[7] = (_Float16)0.0f;
    return f;
}

// LUT entry for byte b: features [n>=1, n>=2, n>=3, max(n-3,0)/2] of n = b & 15, then of b >> 4,
// times the 2^-e scale
BGX_DEV uint4 lut_entry(uint32_t b, float sc) {
    half8 f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int n = (int)((b >> (4 * t)) & 15u);
        f[4 * t + 0] = (_Float16)(n >= 1 ? sc : 0.0f);
        f[4 * t + 1] = (_Float16)(n >= 2 ? sc : 0.0f);
        f[4 * t + 2] = (_Float16)(n >= 3 ? sc : 0.0f);
        f[4 * t + 3] = (_Float16)(n > 3 ? (float)(n - 3) * 0.5f * sc : 0.0f);
    }
    return *(const uint4*)&f;
}

// One 32-board tile through the MLP on one wavefront (the mlp_kernel<1, NW>
// sequence: same MFMA order, same epilogue order, so the same bits). bx / by =
// the packed board of column (lane & 31) (zeros for padding columns); wf / lut
// / w2s = the LDS-resident W fragments, feature LUT and value-head weights.
// Returns w2 . sigmoid(W1 x + b1) for the lane's column (both lane halves
// hold it); the caller adds b2.
BGX_DEV float mlp_tile_value(const uint4* wf, const uint4* lut, const float* w2s, float fs, uint4 bx, uint4 by) {
    const int lane = (int)(threadIdx.x & 63);
    const int h = lane >> 5;
    floatx16 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][r] = 0.0f;
    uint4 ch = wf[((0 * 4 + 0) * KSTEPS + 0) * 64 + lane];
    uint4 cl = wf[((1 * 4 + 0) * KSTEPS + 0) * 64 + lane];
    half8 b = feat_frag(bx, by, 0, h, lut, fs);
#pragma unroll 1
    for (int s = 0; s < KSTEPS; ++s) {
        const int sn = s + 1 < KSTEPS ? s + 1 : s;
        const half8 nb = feat_frag(bx, by, sn, h, lut, fs);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int s2 = m < 3 ? s : sn, m2 = m < 3 ? m + 1 : 0;
            const uint4 nh = wf[((0 * 4 + m2) * KSTEPS + s2) * 64 + lane];
            const uint4 nl = wf[((1 * 4 + m2) * KSTEPS + s2) * 64 + lane];
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ch, b, acc[m], 0, 0, 0);
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&cl, b, acc[m], 0, 0, 0);
            ch = nh;
            cl = nl;
        }
        b = nb;
    }
    float v = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 c4 = *(const float4*)(w2s + 32 * m + 8 * g + 4 * h);
            const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = 4 * g + k;
                const float ex = __builtin_amdgcn_exp2f(acc[m][r]);
                v = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), v);
                if ((r & 1) == 1) __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    return v + __shfl_xor(v, 32, 64);
}

// mlp_tile_value with one m-tile (32 hidden rows) at a time: 16 accumulator
// registers instead of 64 (for the fused lane kernel's 128-register budget).
// The per-(m, column) MFMA chain (k-steps 0..12, hi then lo) and the epilogue
// order (m, then r) are those of mlp_tile_value, so the result has the same bits.
BGX_DEV float mlp_tile_value_m(const uint4* wf, const uint4* lut, const float* w2s, float fs, uint4 bx, uint4 by) {
    const int lane = (int)(threadIdx.x & 63);
    const int h = lane >> 5;
    float v = 0.0f;
#pragma unroll 1
    for (int m = 0; m < 4; ++m) {
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        uint4 ch = wf[((0 * 4 + m) * KSTEPS + 0) * 64 + lane];
        uint4 cl = wf[((1 * 4 + m) * KSTEPS + 0) * 64 + lane];
        half8 b = feat_frag(bx, by, 0, h, lut, fs);
#pragma unroll 1
        for (int s = 0; s < KSTEPS; ++s) {
            const int sn = s + 1 < KSTEPS ? s + 1 : s;
            const uint4 nh = wf[((0 * 4 + m) * KSTEPS + sn) * 64 + lane];
            const uint4 nl = wf[((1 * 4 + m) * KSTEPS + sn) * 64 + lane];
            const half8 nb = feat_frag(bx, by, sn, h, lut, fs);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ch, b, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&cl, b, acc, 0, 0, 0);
            ch = nh;
            cl = nl;
            b = nb;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 c4 = *(const float4*)(w2s + 32 * m + 8 * g + 4 * h);
            const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float ex = __builtin_amdgcn_exp2f(acc[4 * g + k]);
                v = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), v);
            }
        }
    }
    return v + __shfl_xor(v, 32, 64);
}

}  // namespace bgx
