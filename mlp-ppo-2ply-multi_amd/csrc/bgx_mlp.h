// bgx_mlp.h — K3 device code (split-fp16 fragments, fused feature build), shared by
// the MLP kernels (bgx_mlp.hip) and the fused 1-ply lane kernel (bgx_fused.hip).
// Numerics and layout: see the header comment of bgx_mlp.hip.
#pragma once
#include "bgx_device.h"
#include "bgx_kernels.h"

#ifndef BGX_TILE_PF
#define BGX_TILE_PF 1      // > 0: mlp_tile4 reads its A fragments this many MFMA pairs ahead (0: the compiler's schedule; A/B)
#endif
#ifndef BGX_TILE_PRIO
#define BGX_TILE_PRIO 1    // mlp_tile4 issues its MFMA chain at this wave priority (s_setprio; 0: none; A/B)
#endif
#ifndef BGX_TILE_PRIO_EPI
#define BGX_TILE_PRIO_EPI 0   // 1: the priority holds through the epilogue (exp / rcp) too (A/B)
#endif
#ifndef BGX_TILE_NOSKIP
#define BGX_TILE_NOSKIP 1   // 1: mlp_tile4 runs every k-step (straight-line code); 0: zero k-steps skipped (A/B builds;
                            // only the BGX_TILE_PF=0 form has the skip, so NOSKIP=0 needs TILE_PF=0)
#endif
#if BGX_TILE_PF && !BGX_TILE_NOSKIP
#error "BGX_TILE_NOSKIP=0 (zero k-steps skipped) exists only in the BGX_TILE_PF=0 tile; build with -DBGX_TILE_PF=0"
#endif

namespace bgx {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
// LDS-address-space views: reads through them take a ds_read immediate offset
// from one base register (a generic pointer would go through flat loads)
typedef __attribute__((address_space(3))) const v4u* lds_u4p;
typedef __attribute__((address_space(3))) const float* lds_fp;

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

// Nonzero k-steps of a 32-board tile: k-step s < 12 covers the four point
// slots in half (s & 1) of packed word s >> 1; a k-step whose slots are empty
// on every board of the tile has an all-zero B fragment, and the MFMA of a zero
// fragment adds exact zeros, so skipping it leaves the accumulator's bits
// unchanged. k-step 12 (bars, borne-off, side to move, bias) always runs.
BGX_DEV uint32_t tile_kmask(uint4 bx, uint4 by) {
    const uint32_t wd[6] = {bx.x, bx.y, bx.z, bx.w, by.x, by.y};
    uint32_t m = 1u << 12;
#pragma unroll
    for (int s = 0; s < 12; ++s) {
        const uint32_t half = (wd[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
        m |= ballot(half != 0u) ? 1u << s : 0u;
    }
    return m;
}

// Epilogue order (every MLP kernel sums V the same way, so a row's V has the
// same bits whichever kernel, tile or wave computes it): lane half h of column
// c holds 16 hidden rows of each m-tile; p_m = fma chain over those rows
// (r = 0..15) from 0, v_h = ((p_0 + p_1) + p_2) + p_3, V = (v_h + v_(1-h)) + b2.
//
// One (32-board tile, m-tile) item on one wavefront: the MFMA chain over the
// tile's nonzero k-steps (tile_kmask; ascending, hi then lo) and the partial
// p_m of the lane's column half. 16 accumulator registers.
BGX_DEV float mlp_item(const uint4* wf, const uint4* lut, const float* w2s, float fs, uint4 bx, uint4 by,
                       uint32_t kmask, int m) {
    const int lane = (int)(threadIdx.x & 63);
    const int h = lane >> 5;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    // k-steps fully unrolled, fragments of step s in slot s % 3, loaded two
    // steps ahead; zero k-steps (uniform mask bits) skip their MFMAs
    uint4 ah[3], al[3];
    half8 b[3];
    auto load = [&](int s) {
        ah[s % 3] = wf[((0 * 4 + m) * KSTEPS + s) * 64 + lane];
        al[s % 3] = wf[((1 * 4 + m) * KSTEPS + s) * 64 + lane];
        b[s % 3] = feat_frag(bx, by, s, h, lut, fs);
    };
    load(0);
    load(1);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        if (s + 2 < KSTEPS) load(s + 2);
        if (kmask & (1u << s)) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ah[s % 3], b[s % 3], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&al[s % 3], b[s % 3], acc, 0, 0, 0);
        }
    }
    float p = 0.0f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 c4 = *(const float4*)(w2s + 32 * m + 8 * g + 4 * h);
        const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float ex = __builtin_amdgcn_exp2f(acc[4 * g + k]);
            p = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), p);
        }
    }
    return p;
}

// mlp_item over two 32-board tiles at once (same m-tile): each A fragment
// read from LDS feeds both tiles' MFMAs. kmask = the union of the two tiles'
// masks (a k-step that is zero for one tile adds exact zeros to it). p0 / p1
// are the partials of the lane's column in tile 0 / 1.
BGX_DEV void mlp_item2(const uint4* wf, const uint4* lut, const float* w2s, float fs, uint4 bx0, uint4 by0,
                       uint4 bx1, uint4 by1, uint32_t kmask, int m, float& p0, float& p1) {
    const int lane = (int)(threadIdx.x & 63);
    const int h = lane >> 5;
    floatx16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        acc0[r] = 0.0f;
        acc1[r] = 0.0f;
    }
    uint4 ah[3], al[3];
    half8 b0[3], b1[3];
    auto load = [&](int s) {
        ah[s % 3] = wf[((0 * 4 + m) * KSTEPS + s) * 64 + lane];
        al[s % 3] = wf[((1 * 4 + m) * KSTEPS + s) * 64 + lane];
        b0[s % 3] = feat_frag(bx0, by0, s, h, lut, fs);
        b1[s % 3] = feat_frag(bx1, by1, s, h, lut, fs);
    };
    load(0);
    load(1);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        if (s + 2 < KSTEPS) load(s + 2);
        if (kmask & (1u << s)) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ah[s % 3], b0[s % 3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&ah[s % 3], b1[s % 3], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&al[s % 3], b0[s % 3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&al[s % 3], b1[s % 3], acc1, 0, 0, 0);
        }
    }
    float q0 = 0.0f, q1 = 0.0f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 c4 = *(const float4*)(w2s + 32 * m + 8 * g + 4 * h);
        const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float e0 = __builtin_amdgcn_exp2f(acc0[4 * g + k]), e1 = __builtin_amdgcn_exp2f(acc1[4 * g + k]);
            q0 = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + e0), q0);
            q1 = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + e1), q1);
        }
    }
    p0 = q0;
    p1 = q1;
}

// One 32-board tile through all four m-tiles on one wavefront (the fused
// kernel's MLP items): a k-step's feature fragment is built once and feeds its
// eight MFMAs (four m-tiles x hi / lo), and V is complete in the wave, in the
// canonical epilogue order (p_m per m-tile, v_h = ((p_0 + p_1) + p_2) + p_3,
// V = (v_0 + v_1) + b2 on the lanes of half 0), so it has the bits of every
// other MLP kernel. kmask: the tile's nonzero k-steps (tile_kmask). Returns
// v_0 + v_1 (the caller adds b2) on lanes 0..31.
// Fragments are read through two LDS bases (hi terms, lo terms) with
// constant offsets below 64 KB; the asm hides the bases from the compiler,
// which would otherwise fold them into one base plus an address add per read
// (the fragments sit past the 64 KB an immediate offset reaches).
template <bool STAMP = false>
BGX_DEV float mlp_tile4(const uint4* wf, const uint4* lut, const float* w2s, float fs, uint4 bx, uint4 by,
                        uint32_t kmask, unsigned long long* stamp = nullptr) {
    const int lane = (int)(threadIdx.x & 63);
    const int h = lane >> 5;
    lds_u4p wfh = (lds_u4p)(wf + lane);
    lds_u4p wfl = (lds_u4p)(wf + 4 * KSTEPS * 64 + lane);
    lds_fp w2h = (lds_fp)(w2s + 4 * h);
    asm volatile("" : "+v"(wfh));
    asm volatile("" : "+v"(wfl));
    asm volatile("" : "+v"(w2h));
    floatx16 acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][r] = 0.0f;
#if BGX_TILE_PF
    // Software-pipelined fragment reads: the 52 (k-step, m-tile) pairs of A
    // fragments (hi, lo) run through a ring of BGX_TILE_PF + 1 register pairs,
    // read BGX_TILE_PF pairs ahead of their MFMAs, and the next k-step's feature
    // fragment one m-tile round ahead. Left to itself the compiler issued each
    // pair's two ds_read_b128 right before its MFMAs and waited for them there
    // (lgkmcnt(1) / (0) before every MFMA), so each MFMA paid the LDS latency;
    // the sched_barrier keeps the early reads in front. Same MFMAs in the same
    // order on each accumulator: same bits.
    constexpr int NP = 4 * KSTEPS, D = BGX_TILE_PF, NR = D + 1;
    v4u ra[NR], rl[NR];
    half8 rb[2];
    auto ld = [&](int i) {
        const int s = i >> 2, m = i & 3;
        ra[i % NR] = wfh[(m * KSTEPS + s) * 64];
        rl[i % NR] = wfl[(m * KSTEPS + s) * 64];
    };
    rb[0] = feat_frag(bx, by, 0, h, lut, fs);
#pragma unroll
    for (int i = 0; i < D; ++i) ld(i);
    if (BGX_TILE_PRIO) __builtin_amdgcn_s_setprio(BGX_TILE_PRIO);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int s = i >> 2, m = i & 3;
        if (i + D < NP) ld(i + D);
        if (m == 0 && s + 1 < KSTEPS) rb[(s + 1) & 1] = feat_frag(bx, by, s + 1, h, lut, fs);
        __builtin_amdgcn_sched_barrier(0);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ra[i % NR]), rb[s & 1], acc[m], 0, 0, 0);
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, rl[i % NR]), rb[s & 1], acc[m], 0, 0, 0);
    }
    if (BGX_TILE_PRIO && !BGX_TILE_PRIO_EPI) __builtin_amdgcn_s_setprio(0);
    (void)kmask;
#else
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        if (BGX_TILE_NOSKIP || (kmask & (1u << s))) {
            const half8 b = feat_frag(bx, by, s, h, lut, fs);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const v4u ah = wfh[(m * KSTEPS + s) * 64];
                const v4u al = wfl[(m * KSTEPS + s) * 64];
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, ah), b, acc[m], 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, al), b, acc[m], 0, 0, 0);
            }
        }
    }
#endif
    if (STAMP) *stamp = wall_clock64();   // development (BGX_FUSED_PROF): the MFMA chain issued
    float v = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float p = 0.0f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            // (read as a float vector: hipcc 7.2 miscompiles bit_cast of the
            // lanes of a u32 vector loaded from LDS -- every lane became .x)
            const v4f c4 = *(__attribute__((address_space(3))) const v4f*)(w2h + 32 * m + 8 * g);
            const float cy[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float ex = __builtin_amdgcn_exp2f(acc[m][4 * g + k]);
                p = fmaf(cy[k], __builtin_amdgcn_rcpf(1.0f + ex), p);
            }
        }
        v = m == 0 ? p : v + p;
    }
#if BGX_TILE_PF
    if (BGX_TILE_PRIO && BGX_TILE_PRIO_EPI) __builtin_amdgcn_s_setprio(0);
#endif
    return v + __shfl_xor(v, 32, 64);
}

}  // namespace bgx
