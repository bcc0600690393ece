// bgx_domain.h — the input domain of the stateless entry points (include/bgx.h,
// BGX_BADF_*), one function shared by the device check (validate_kernel,
// bgx_encode.hip) and the host variant bgx_check_boards_host (bgx_abi.cpp).
//
// The reference's ImmutableBoard holds per-point counts for each player
// (board/immutable_board.py:16-24) with at most 15 checkers a side, and no
// point is held by both players in a reachable position; dice come from
// np.random.randint(1, 7) (environments/backgammon_env.py:310-311).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bgx.h"

namespace bgx {

// b: u8[52] board (4-byte aligned), player: 0/1 or < 0 = unchecked, dice:
// u8[2] or null = unchecked. Returns the BGX_BADF_* bits the input violates.
__host__ __device__ inline unsigned domain_bits(const uint8_t* b, int player, const uint8_t* dice) {
    uint32_t t[13];
    for (int k = 0; k < 13; ++k)
        t[k] = (uint32_t)b[4 * k] | (uint32_t)b[4 * k + 1] << 8 | (uint32_t)b[4 * k + 2] << 16 |
               (uint32_t)b[4 * k + 3] << 24;
    unsigned bad = 0, sum0 = 0, sum1 = 0;
    for (int k = 0; k < 13; ++k) {
        if (t[k] & 0xF0F0F0F0u) bad |= BGX_BADF_VALUE;   // a byte above 15
        for (int q = 0; q < 4; ++q) {
            const unsigned v = (t[k] >> (8 * q)) & 0xFFu;
            const int idx = 4 * k + q;   // p0 0..23 | p1 24..47 | bar1 48, bar2 49 | off1 50, off2 51
            if (idx < 24 || idx == 48 || idx == 50) sum0 += v;
            else sum1 += v;
        }
    }
    // a point held by both: byte-wise nonzero masks of p0[0..23] and p1[0..23]
    for (int k = 0; k < 6; ++k) {
        const uint32_t a = t[k], c = t[6 + k];
        const uint32_t na = (((a & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | a) & 0x80808080u;
        const uint32_t nc = (((c & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | c) & 0x80808080u;
        if (na & nc) bad |= BGX_BADF_SHARED_POINT;
    }
    if (sum0 > 15 || sum1 > 15) bad |= BGX_BADF_TOTAL;
    if (player > 1) bad |= BGX_BADF_PLAYER;
    if (dice) {
        const unsigned d0 = dice[0], d1 = dice[1];
        if (d0 < 1 || d0 > 6 || d1 < 1 || d1 > 6) bad |= BGX_BADF_DICE;
    }
    return bad;
}

}  // namespace bgx
