// tests/cpuwave/mlp_emu.cpp -- test infrastructure (host build, emulated workgroups).
// The MLP launch (bgx_launch_mlp, bgx_mlp.hip: LUT feature build, split-fp16
// MFMA tiles, canonical epilogue) on the host: the kernels' source (a copy
// with the inline-asm scheduling hints removed and the dynamic LDS array
// bound to the emulated workgroup's buffer) against
// tests/cpuwave/hip/hip_runtime.h, whose v_mfma_f32_32x32x16_f16 follows the
// operand layout the fragments are built for (bgx_frag.h).
// Usage: mlp_emu rows.bin weights.bin nt out.bin [roots.bin]
//   rows: n x 8 packed words (uint32); weights: W1 [128][198], b1 [128],
//   w2 [128], b2 [1] (float32); nt 1 or 2 (the launcher's two kernels), or d:
//   the 2-ply replies by difference (the root launch with zout over roots.bin,
//   then mlp_kernel_delta over rows whose word 7 is the root's index);
//   out: n float32 V
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bgx_frag.h"
#include "bgx_mlp.hip"

static_assert(bgx_frag::NFRAG == bgx::NFRAG, "fragment count");

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    std::vector<uint32_t> rows;
    {
        FILE* f = fopen(argv[1], "rb");
        if (!f) return 2;
        uint32_t v[8];
        while (fread(v, 4, 8, f) == 8) rows.insert(rows.end(), v, v + 8);
        fclose(f);
    }
    std::vector<float> w(128 * 198 + 128 + 128 + 1);
    {
        FILE* f = fopen(argv[2], "rb");
        if (!f || fread(w.data(), 4, w.size(), f) != w.size()) return 2;
        fclose(f);
    }
    const float* W1 = w.data();
    const float* b1 = W1 + 128 * 198;
    const float* w2 = b1 + 128;
    const float b2 = w2[128];
    std::vector<uint16_t> frag;
    const int e = bgx_frag::build_fragments(W1, b1, frag);
    const int n = (int)rows.size() / 8;
    std::vector<float> out(n, -12345.0f);
    bgx::MlpArgs a{};
    a.rows = rows.data();
    a.n_rows = n;
    a.n_max = n;
    const bool delta = argv[3][0] == 'd';
    a.nt = delta ? 2 : atoi(argv[3]);
    a.out = out.data();
    a.wfrag = (const uint4*)frag.data();
    a.rowc = w2;
    a.b2 = b2;
    a.feat_scale = (float)std::ldexp(1.0, -e);
    std::vector<uint32_t> roots;
    std::vector<float> zt, vr;
    if (delta) {
        if (argc < 6) return 2;
        FILE* f = fopen(argv[5], "rb");
        if (!f) return 2;
        uint32_t v[8];
        while (fread(v, 4, 8, f) == 8) roots.insert(roots.end(), v, v + 8);
        fclose(f);
        const int nr = (int)roots.size() / 8;
        zt.assign((size_t)nr * 128, -777.0f);
        vr.assign(nr, 0.0f);
        bgx::MlpArgs m = a;
        m.rows = roots.data();
        m.n_rows = nr;
        m.n_max = nr;
        m.nt = 1;
        m.out = vr.data();
        m.zout = zt.data();
        m.z_base = 0;
        if (bgx_launch_mlp(&m, nullptr) != hipSuccess) return 3;
        a.zt = zt.data();
        a.root_rows = roots.data();
        a.root_sel = nullptr;
        a.root_base = 0;
        a.n_roots = nr;
        a.n_slots = nr;
    }
    if (bgx_launch_mlp(&a, nullptr) != hipSuccess) return 3;
    FILE* f = fopen(argv[4], "wb");
    if (!f) return 2;
    fwrite(out.data(), 4, out.size(), f);
    fclose(f);
    return 0;
}
