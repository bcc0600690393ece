// tests/cpuwave/reply_emu.cpp -- test infrastructure (host build, emulated workgroups).
// The 2-ply reply launch exactly as bgx_reply_moves issues it (bgx_movegen.hip
// compiled for the host against tests/cpuwave/hip/hip_runtime.h: the reply
// kernel's 16-wave workgroups, its sub-queue and per-roll calls, then the
// tier-2 block kernel), on candidate rows from a file, with exact-size
// buffers under AddressSanitizer. Writes every job's record count and rows
// (in order) to the dump file, so two launch forms (BGX_REPLY_DBL=0 / 1) can be
// compared byte for byte.
// Usage: reply_emu positions.bin n_roots dump.bin   (positions: 8 packed words + mover, int32)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bgx_movegen.hip"

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    setvbuf(stdout, nullptr, _IONBF, 0);
    setenv("BGX_MG_FEW", "0", 1);   // the pool / reply kernels, as the engine's large launches
    const int n_max = atoi(argv[2]);
    std::vector<uint32_t> rows;
    {
        FILE* f = fopen(argv[1], "rb");
        if (!f) return 2;
        uint32_t v[9];
        int n = 0;
        while (n < n_max && fread(v, 4, 9, f) == 9) {
            rows.insert(rows.end(), v, v + 8);
            ++n;
        }
        fclose(f);
    }
    const int n = (int)rows.size() / 8;
    const int n_jobs = n * 21, cap = n * 21 * 64 + 4096;
    const int ws_waves = 64, ws_slots = 16384, ovf_cap = 1 << 16;
    std::vector<uint32_t> out((size_t)cap * 8, 0xDEADBEEFu), ws((size_t)ws_waves * 5 * ws_slots, 0u);
    std::vector<int32_t> off(n_jobs, -7), cnt(n_jobs, -7), ovf(ovf_cap, 0);
    std::vector<unsigned> ctr(8, 0u);
    bgx::MovegenArgs b{};
    b.n_jobs = n_jobs;
    b.in_mode = bgx::IN_TWOPLY;
    b.in_packed = rows.data();
    b.out_mode = bgx::OUT_PACKED_FLAT;
    b.out_packed = out.data();
    b.flat_count = ctr.data();
    b.flat_cap = cap;
    b.flat_chunk = 256;
    b.job_off = off.data();
    b.job_cnt = cnt.data();
    b.ovf_count = ctr.data() + 2;
    b.ovf_list = ovf.data();
    b.ovf_cap = ovf_cap;
    b.ws_global = ws.data();
    b.ws_waves = ws_waves;
    b.ws_slots = ws_slots;
    b.ws_words_per_wave = (size_t)5 * ws_slots;
    b.err_flags = ctr.data() + 3;
    if (bgx_launch_movegen(&b, nullptr) != hipSuccess) return 3;
    // job_off / job_cnt start poisoned (-7): every job of the launch must write both
    int unwritten = 0;
    for (int j = 0; j < n_jobs; ++j) unwritten += off[j] == -7 || cnt[j] == -7;
    printf("{\"roots\": %d, \"rows\": %u, \"tier2_jobs\": %u, \"flags\": %u, \"unwritten_jobs\": %d}\n", n, ctr[0],
           ctr[2], ctr[3], unwritten);
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 2;
    for (int j = 0; j < n_jobs; ++j) {
        fwrite(&cnt[j], 4, 1, f);
        if (cnt[j] > 0 && off[j] >= 0 && (size_t)off[j] + cnt[j] <= (size_t)cap)
            fwrite(out.data() + (size_t)off[j] * 8, 4, (size_t)cnt[j] * 8, f);
    }
    fclose(f);
    return ctr[3] ? 4 : (unwritten ? 5 : 0);
}
