// tests/cpuwave/dbl_check.cpp -- test infrastructure (host build, emulated wave).
// Board-major doubles (board_dbl_emit, bgx_movegen.h) against the per-roll
// path (run_job<false, true>: path_doubles_emit / job_records) on random
// positions: for every (root, die) the same record count and the same rows in
// the same order; every write inside its job's reserved rows (the output
// buffer has exact size and guard rows, and the build runs under
// AddressSanitizer, so a stray LDS or output access aborts with a report).
// Usage: dbl_check [n_roots] [seed] [positions.bin: per root 8 packed words + mover, int32]
//   -> one summary line, exit 0 iff clean. -DEMU_TRACE: report where the lanes wait (a harness
//   whose lanes reach different cross-lane operations deadlocks).
#include <chrono>
#include <cstdio>
#include <unistd.h>
#include <cstdlib>
#include <random>
#include <vector>

#include "bgx_movegen.h"

using namespace bgx;

namespace {
constexpr int P_S = 256, P_F = 224, P_PF = 480, SLICE_WORDS = 64 + 2 * P_PF;   // the reply kernel's slice
constexpr int GUARD = 64;                                                        // rows past flat_cap
constexpr uint32_t SENT = 0xDEADBEEFu;

struct Out {
    std::vector<uint32_t> rows;   // (cap + GUARD) x 8
    int32_t off[21], cnt[21];
    unsigned count = 0, err = 0;
};

struct Shared {
    MovegenArgs a{};
    Mem M{};
    uint32_t* slice = nullptr;
    uint32_t cntd[8];
    int ref_r[7];
    uint32_t rest = 0;
} S;

void setup_args(Out& o, int cap) {
    o.rows.assign((size_t)(cap + GUARD) * 8, SENT);
    for (int i = 0; i < 21; ++i) o.off[i] = o.cnt[i] = -7;
    o.count = 0;
    o.err = 0;
    MovegenArgs& a = S.a;
    a = MovegenArgs{};
    a.n_jobs = 21;
    a.in_mode = IN_TWOPLY;
    a.out_mode = OUT_PACKED_FLAT;
    a.out_packed = o.rows.data();
    a.flat_count = &o.count;
    a.flat_cap = cap;
    a.flat_chunk = 64;
    a.job_off = o.off;
    a.job_cnt = o.cnt;
    a.err_flags = &o.err;
    a.heavy_t = 0x7FFFFFFF;
}

// a random position: the mover's 15 checkers (bar / off / points), the
// opponent's on points the mover does not hold
void random_board(std::mt19937& g, uint32_t* w, int& player) {
    int c[2][24] = {}, bar[2] = {0, 0}, off[2] = {0, 0};
    player = (int)(g() & 1u);
    for (int p = 0; p < 2; ++p) {
        int left = 15;
        const int r = (int)(g() % 10u);
        bar[p] = r == 0 ? 1 : (r == 1 ? 2 : 0);
        left -= bar[p];
        off[p] = (g() % 6u) == 0 ? (int)(g() % 4u) : 0;
        left -= off[p];
        while (left > 0) {
            const int q = (int)(g() % 24u);
            if (c[1 - p][q]) continue;
            const int k = 1 + (int)(g() % (unsigned)std::min(left, 4));
            c[p][q] += k;
            left -= k;
        }
    }
    for (int i = 0; i < 8; ++i) w[i] = 0;
    for (int p = 0; p < 2; ++p)
        for (int q = 0; q < 24; ++q) w[3 * p + (q >> 3)] |= (uint32_t)c[p][q] << (4 * (q & 7));
    w[6] = (uint32_t)bar[0] | (uint32_t)bar[1] << 4 | (uint32_t)off[0] << 8 | (uint32_t)off[1] << 12 |
           (uint32_t)(1 - player) << 16;
}
}  // namespace

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int n_roots = argc > 1 ? atoi(argv[1]) : 300;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1u;
    std::vector<uint32_t> slice(SLICE_WORDS, 0u);
    S.slice = slice.data();
    Mem& M = S.M;
    M.map = S.slice;
    M.tab = (unsigned long long*)(S.slice + 64);
    M.S = P_S;
    M.F = P_F;
    M.fa = S.slice + 64 + 2 * P_S;
    M.fb = M.fa + P_F;
    M.pa = S.slice + 64;
    M.pb = M.pa + P_PF;
    M.PF = P_PF;
    const int cap = 21 * 2048;
    Out ref, bm;
    long long n_jobs = 0, n_rows = 0, n_tier2 = 0, n_bm_roots = 0, n_rest = 0, bad = 0;
    std::barrier<> barrier(64);
    emu::bar = &barrier;
    std::mt19937 g(seed);
    std::vector<std::vector<uint32_t>> boards(n_roots, std::vector<uint32_t>(8));
    std::vector<int> players(n_roots);
    for (int i = 0; i < n_roots; ++i) random_board(g, boards[i].data(), players[i]);
    if (argc > 3) {   // positions from a file: per root 8 packed words + the mover (int32 x 9)
        FILE* f = fopen(argv[3], "rb");
        if (!f) return 2;
        std::vector<int32_t> buf;
        int32_t v[9];
        boards.clear();
        players.clear();
        while (fread(v, 4, 9, f) == 9 && (int)boards.size() < n_roots) {
            boards.emplace_back(v, v + 8);
            players.push_back(v[8]);
        }
        fclose(f);
    }
    const int n_cases = (int)boards.size();

    auto lane_main = [&](int lane) {
        emu::lane = lane;
        emu::tid = lane;
        for (int i = 0; i < n_cases; ++i) {
            // the jobs in every lane's registers (make_job reads lanes: all lanes run it)
            JobIn in[7];
            {
                const uint32_t* w = boards[i].data();
                for (int d = 0; d <= 6; ++d)
                    in[d] = make_job(w[0], w[1], w[2], w[3], w[4], w[5], w[6], players[i], d ? d : 1, d ? d : 1);
            }
            if (lane == 0) setup_args(ref, cap);
            emu::sync();
            // the per-roll path: six (d, d) jobs
            {
                FlatCursor fc;
                fc.left_hint = 6;
                for (int d = 1; d <= 6; ++d) {
                    const int r = run_job<false, true>(S.a, dbl_q21(d), in[d], S.M, fc);
                    if (lane == 0) S.ref_r[d] = r;
                }
            }
            emu::sync();
            if (lane == 0) setup_args(bm, cap);
            emu::sync();
            // the row's non-doubles item first, as the reply kernel runs it on the
            // same slice (it must leave the parent map zero)
            {
                int rc = 0;
                const int n_nd = board_nd_records2<P_PF>(in[1].R, S.M.map, S.M.pa, S.M.pb, rc);
                (void)n_nd;
                emu::sync();
                if (lane == 0)
                    for (int q = 0; q < 64; ++q)
                        if (S.slice[q]) {
                            printf("root %d: board_nd_records2 left map[%d] = %u (n %d)\n", i, q, S.slice[q], n_nd);
                            ++bad;
                            break;
                        }
                emu::sync();
            }
            // board-major: one item, the dice it leaves run per roll
            {
                FlatCursor fc;
                fc.left_hint = 6;
                const uint32_t rest = board_dbl_emit<false>(S.a, 0, in[0], S.M, fc, S.cntd);
                if (lane == 0) S.rest = rest;
                for (int d = 1; d <= 6; ++d)
                    if ((rest >> (d - 1)) & 1u) run_job<false, true>(S.a, dbl_q21(d), in[d], S.M, fc);
            }
            emu::sync();
            if (lane == 0) {
                for (int q = 0; q < 64; ++q)
                    if (S.slice[q]) {
                        printf("root %d: map[%d] = %u after the doubles\n", i, q, S.slice[q]);
                        ++bad;
                        break;
                    }
                n_bm_roots += S.rest != 0x3Fu;
                n_rest += __builtin_popcount(S.rest);
                if (bm.err || ref.err) {
                    printf("root %d: error flags ref 0x%x board-major 0x%x\n", i, ref.err, bm.err);
                    ++bad;
                }
                for (int d = 1; d <= 6; ++d) {
                    const int j = dbl_q21(d);
                    ++n_jobs;
                    if (S.ref_r[d] < 0) {
                        ++n_tier2;
                        continue;
                    }
                    if (ref.cnt[j] != bm.cnt[j]) {
                        printf("root %d die %d: count ref %d board-major %d (rest 0x%x)\n", i, d, ref.cnt[j], bm.cnt[j],
                               S.rest);
                        ++bad;
                        continue;
                    }
                    n_rows += ref.cnt[j];
                    for (int k = 0; k < ref.cnt[j]; ++k)
                        for (int q = 0; q < 8; ++q)
                            if (ref.rows[(size_t)(ref.off[j] + k) * 8 + q] != bm.rows[(size_t)(bm.off[j] + k) * 8 + q]) {
                                printf("root %d die %d: row %d word %d differs\n", i, d, k, q);
                                ++bad;
                                k = ref.cnt[j];
                                break;
                            }
                }
                // nothing written past the reserved rows
                for (size_t r = bm.count; r < (size_t)cap + GUARD; ++r)
                    if (bm.rows[r * 8] != SENT) {
                        printf("root %d: row %zu written past the reservations (%u)\n", i, r, bm.count);
                        ++bad;
                        break;
                    }
            }
            emu::sync();
        }
    };
#ifdef EMU_TRACE
    std::thread([&] {
        std::this_thread::sleep_for(std::chrono::seconds(8));
        for (int l = 0; l < 64; l += 1) {
            printf("lane %d syncs %llu:", l, emu::nsync[l]);
            for (int k = 0; k < emu::nwhere[l]; ++k) printf(" %p", emu::where[l][k]);
            printf("\n");
        }
        fflush(stdout);
        _exit(3);
    }).detach();
#endif
    std::vector<std::thread> th;
    for (int l = 0; l < 64; ++l) th.emplace_back(lane_main, l);
    for (auto& t : th) t.join();
    printf("{\"roots\": %d, \"jobs\": %lld, \"rows\": %lld, \"tier2_jobs\": %lld, \"board_major_roots\": %lld, "
           "\"dice_left_to_per_roll\": %lld, \"mismatches\": %lld}\n",
           n_cases, n_jobs, n_rows, n_tier2, n_bm_roots, n_rest, bad);
    return bad ? 1 : 0;
}
