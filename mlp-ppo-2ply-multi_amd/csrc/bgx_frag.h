// bgx_frag.h — host side of the split-fp16 MLP: W1 / b1 -> the MFMA A
// fragments the MLP kernels keep in LDS (scheme: bgx_mlp.hip header). Used by
// bgx_set_weights (bgx_abi.cpp) and the host emulation tests (tests/cpuwave/).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

// (the same constants as bgx_mlp.h's KSTEPS / NFRAG, which this host header
// does not include: it is also compiled into the ABI translation unit)
namespace bgx_frag {

constexpr int KSTEPS = 13;                   // 208 = 13 x 16 >= 198 features
constexpr int NFRAG = 2 * 4 * KSTEPS * 64;   // 16-byte fragments

// Split-fp16 fragments (see bgx_mlp.hip header for the scheme). Returns e.
inline constexpr double kLog2e = 1.4426950408889634;

inline int build_fragments(const float* W1, const float* b1, std::vector<uint16_t>& frag) {
    std::vector<double> Wp(128 * 208, 0.0);
    double mx = 0.0;
    for (int j = 0; j < 128; ++j) {
        for (int k = 0; k < 198; ++k) {
            double v = W1[j * 198 + k];
            if (k == 193 || k == 195) v /= 15.0;   // feature = integer borne-off count
            Wp[j * 208 + k] = -kLog2e * v;          // accumulator = -h log2(e): sigmoid = 1 / (1 + 2^acc)
        }
        Wp[j * 208 + 198] = -kLog2e * b1[j];       // bias column, constant feature
        for (int k = 0; k < 208; ++k) mx = std::fmax(mx, std::fabs(Wp[j * 208 + k]));
    }
    // W scaled by 2^e (largest |w| in [2^14, 2^15)), features by 2^-e; e <= 13
    // keeps the smallest feature (0.5 * 2^-e) a normal fp16, e >= -11 keeps the
    // largest (15 * 2^-e) finite
    int e = 0;
    if (mx > 0.0) {
        e = 14 - (int)std::floor(std::log2(mx));
        if (e > 13) e = 13;
        if (e < -11) e = -11;
    }
    const double sc = std::ldexp(1.0, e);
    std::vector<_Float16> hi(128 * 208), lo(128 * 208);
    for (int i = 0; i < 128 * 208; ++i) {
        const double x = Wp[i] * sc;
        const _Float16 h = (_Float16)(float)x;
        hi[i] = h;
        lo[i] = (_Float16)(float)(x - (double)(float)h);
    }
    frag.assign((size_t)NFRAG * 8, 0);
    for (int t = 0; t < 2; ++t)
        for (int m = 0; m < 4; ++m)
            for (int s = 0; s < KSTEPS; ++s)
                for (int l = 0; l < 64; ++l)
                    for (int jj = 0; jj < 8; ++jj) {
                        const int row = 32 * m + (l & 31);
                        const int k = 16 * s + 8 * (l >> 5) + jj;
                        const _Float16 v = (t == 0 ? hi : lo)[row * 208 + k];
                        uint16_t bits;
                        std::memcpy(&bits, &v, 2);
                        frag[((((size_t)t * 4 + m) * KSTEPS + s) * 64 + l) * 8 + jj] = bits;
                    }
    return e;
}

}  // namespace bgx_frag
