// bgx_device.h — gfx950 device helpers shared by the bgx kernels.
//
// Board representation on the device ("packed board", 32 B, two dwordx4):
//   w[0..2]  PLAYER1 point counts, point i in nibble (i & 7) of w[i >> 3]
//   w[3..5]  PLAYER2 point counts
//   w[6]     bar1 | bar2 << 4 | off1 << 8 | off2 << 12 | flag << 16
//            (flag = the player whose indicator features 196/197 are set;
//             immutable_board.py:122-127)
//   w[7]     reserved (0)
// Counts are 0..15 (15 checkers per side), so a nibble is exact.
//
// Movegen "node" representation (relative to a wave-uniform root):
//   m[0..2] mover point nibbles, x = bar | off << 4 | hits << 8 (24-bit mask of
//   opponent blots hit on this turn). Opponent state = root opponent minus
//   the hit blots (opponent blocks never change during the mover's turn, so
//   they are a per-job constant). The 128-bit (m0,m1,m2,x) is an exact key of
//   the resulting ImmutableBoard for a given root.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BGX_DEV __device__ __forceinline__

namespace bgx {

// ------------------------------------------------------------ Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };

BGX_DEV u32x4 philox(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo) {
    uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
    uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}
BGX_DEV int die_from(uint32_t r) { return 1 + (int)(((uint64_t)r * 6u) >> 32); }
BGX_DEV float unit_from(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

// ------------------------------------------------------------ nibble helpers
// 8 nibbles -> 8-bit "nonzero" mask.
BGX_DEV uint32_t nz8(uint32_t w) {
    uint32_t t = (w | (w >> 1) | (w >> 2) | (w >> 3)) & 0x11111111u;
    t = (t | (t >> 3)) & 0x03030303u;
    t = (t | (t >> 6)) & 0x000F000Fu;
    return (t | (t >> 12)) & 0xFFu;
}
// 8 nibbles -> 8-bit ">= 2" mask.
BGX_DEV uint32_t ge2_8(uint32_t w) {
    uint32_t t = ((w >> 1) | (w >> 2) | (w >> 3)) & 0x11111111u;
    t = (t | (t >> 3)) & 0x03030303u;
    t = (t | (t >> 6)) & 0x000F000Fu;
    return (t | (t >> 12)) & 0xFFu;
}
BGX_DEV uint32_t occ24(uint32_t a, uint32_t b, uint32_t c) {
    return nz8(a) | (nz8(b) << 8) | (nz8(c) << 16);
}
BGX_DEV uint32_t ge2_24(uint32_t a, uint32_t b, uint32_t c) {
    return ge2_8(a) | (ge2_8(b) << 8) | (ge2_8(c) << 16);
}
// sum of the nibbles of w
BGX_DEV uint32_t nibsum(uint32_t w) {
    uint32_t t = (w & 0x0F0F0F0Fu) + ((w >> 4) & 0x0F0F0F0Fu);
    return (t * 0x01010101u) >> 24;
}
// 4 bytes (each <16) -> 4 nibbles (16 bits)
BGX_DEV uint32_t pack4(uint32_t w) {
    return (w & 0xFu) | ((w >> 4) & 0xF0u) | ((w >> 8) & 0xF00u) | ((w >> 12) & 0xF000u);
}
// 8 nibbles -> two words of 4 bytes each
BGX_DEV void unpack8(uint32_t w, uint32_t& lo, uint32_t& hi) {
    lo = (w & 0xFu) | ((w & 0xF0u) << 4) | ((w & 0xF00u) << 8) | ((w & 0xF000u) << 12);
    uint32_t v = w >> 16;
    hi = (v & 0xFu) | ((v & 0xF0u) << 4) | ((v & 0xF00u) << 8) | ((v & 0xF000u) << 12);
}
BGX_DEV uint32_t nib(const uint32_t m0, const uint32_t m1, const uint32_t m2, int i) {
    uint32_t w = i < 8 ? m0 : (i < 16 ? m1 : m2);
    return (w >> ((i & 7) * 4)) & 0xFu;
}

// ------------------------------------------------------------ job root
struct Root {
    uint32_t m0, m1, m2;   // mover nibbles
    uint32_t o0, o1, o2;   // opponent nibbles
    uint32_t bar, off;     // mover bar / off
    uint32_t obar, ooff;   // opponent bar / off
    uint32_t block;        // opponent points with >= 2 checkers
    uint32_t blot;         // opponent points with exactly 1
    int player;            // mover: 0 = PLAYER1, 1 = PLAYER2
};

struct Node { uint32_t m0, m1, m2, x; };

// packed board (8 words) -> root for `player`
BGX_DEV Root make_root(const uint32_t* w, int player) {
    Root r;
    const uint32_t* me = w + 3 * player;
    const uint32_t* op = w + 3 * (1 - player);
    r.m0 = me[0]; r.m1 = me[1]; r.m2 = me[2];
    r.o0 = op[0]; r.o1 = op[1]; r.o2 = op[2];
    uint32_t s = w[6];
    r.bar = (s >> (4 * player)) & 15u;
    r.obar = (s >> (4 * (1 - player))) & 15u;
    r.off = (s >> (8 + 4 * player)) & 15u;
    r.ooff = (s >> (8 + 4 * (1 - player))) & 15u;
    r.block = ge2_24(r.o0, r.o1, r.o2);
    r.blot = occ24(r.o0, r.o1, r.o2) & ~r.block;
    r.player = player;
    return r;
}
BGX_DEV Node root_node(const Root& r) { return {r.m0, r.m1, r.m2, r.bar | (r.off << 4)}; }

// node -> packed board words (w[0..7]) with indicator flag `flag`
// bit i of an 8-bit value -> bit 4i (one bit per nibble)
BGX_DEV uint32_t spread8(uint32_t x) {
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
}

BGX_DEV void node_to_packed(const Root& r, const Node& n, uint32_t flag, uint32_t* w) {
    uint32_t hit = n.x >> 8;
    // zero the opponent nibbles at the hit points (each was exactly 1):
    // spread each hit byte to one bit per nibble
    const uint32_t h0 = spread8(hit & 0xFFu), h1 = spread8((hit >> 8) & 0xFFu), h2 = spread8((hit >> 16) & 0xFFu);
    uint32_t o0 = r.o0 - h0, o1 = r.o1 - h1, o2 = r.o2 - h2;
    uint32_t obar = r.obar + __popc(hit);
    uint32_t bar = n.x & 15u, off = (n.x >> 4) & 15u;
    if (r.player == 0) {
        w[0] = n.m0; w[1] = n.m1; w[2] = n.m2; w[3] = o0; w[4] = o1; w[5] = o2;
        w[6] = bar | (obar << 4) | (off << 8) | (r.ooff << 12) | (flag << 16);
    } else {
        w[0] = o0; w[1] = o1; w[2] = o2; w[3] = n.m0; w[4] = n.m1; w[5] = n.m2;
        w[6] = obar | (bar << 4) | (r.ooff << 8) | (off << 12) | (flag << 16);
    }
    w[7] = 0;
}

// packed -> u8[52] (13 words)
BGX_DEV void packed_to_u8(const uint32_t* w, uint32_t* o) {
#pragma unroll
    for (int k = 0; k < 6; ++k) unpack8(w[k], o[2 * k], o[2 * k + 1]);
    uint32_t s = w[6];
    o[12] = (s & 15u) | (((s >> 4) & 15u) << 8) | (((s >> 8) & 15u) << 16) | (((s >> 12) & 15u) << 24);
}
// u8[52] (13 words) -> packed (flag in w[6])
BGX_DEV void u8_to_packed(const uint32_t* b, uint32_t flag, uint32_t* w) {
#pragma unroll
    for (int k = 0; k < 6; ++k) w[k] = pack4(b[2 * k]) | (pack4(b[2 * k + 1]) << 16);
    uint32_t t = b[12];
    w[6] = (t & 15u) | (((t >> 8) & 15u) << 4) | (((t >> 16) & 15u) << 8) | (((t >> 24) & 15u) << 12) |
           (flag << 16);
    w[7] = 0;
}

// ------------------------------------------------------------ one-die move lists
// A node's ordered SubMove list for one die (get_moves_with_one_die,
// get_moves_one_die.py:13-251) is: the set bits of `src` in ascending point
// order (normal moves; in BEAR_OFF only home points), then up to two bear-off
// sources e0/e1 (farthest checker, exact point), or a single bar entry.
// Sources are point indices 0..23, 24 = BAR; the destination follows from the
// source: P1 s+d (>= 24: bear off), P2 s-d (< 0: bear off), BAR: d-1 / 24-d.
struct Moves {
    uint32_t src;   // ordered normal-move sources
    int nsrc;
    int e0, e1;     // extra sources (bear-off) or 24 (bar entry)
    int n;          // total moves
};

// "destination is on the board and not blocked" masks for die d
BGX_DEV uint32_t ok_mask(uint32_t block, int d, int player) {
    uint32_t free = ~block & 0xFFFFFFu;
    return player == 0 ? (free >> d) & ((1u << (24 - d)) - 1u) : (free << d) & 0xFFFFFFu;
}

BGX_DEV Moves node_moves(const Root& r, const Node& n, int d, uint32_t okd) {
    Moves mv;
    mv.src = 0; mv.nsrc = 0; mv.e0 = -1; mv.e1 = -1; mv.n = 0;
    uint32_t bar = n.x & 15u, off = (n.x >> 4) & 15u;
    if (off == 15u) return mv;                         // GAME_OVER (conditions.py:16-17)
    if (bar > 0u) {                                    // ON_BAR (get_moves_bar)
        int entry = r.player == 0 ? d - 1 : 24 - d;
        if (!((r.block >> entry) & 1u)) { mv.e0 = 24; mv.n = 1; }
        return mv;
    }
    uint32_t occ = occ24(n.m0, n.m1, n.m2);
    const uint32_t home = r.player == 0 ? 0xFC0000u : 0x3Fu;
    uint32_t hsum = r.player == 0 ? nibsum(n.m2 >> 8) : nibsum(n.m0 & 0xFFFFFFu);
    bool bear = ((occ & ~home) == 0u) && (hsum + off == 15u);   // all_checkers_home
    if (!bear) {                                       // NORMAL (get_moves_normal)
        mv.src = occ & okd;
        mv.nsrc = __popc(mv.src);
        mv.n = mv.nsrc;
        return mv;
    }
    // BEAR_OFF (get_moves_bear_off, get_moves_one_die.py:133-251)
    uint32_t oh = occ & home;
    mv.src = oh & okd;
    mv.nsrc = __popc(mv.src);
    mv.n = mv.nsrc;
    int last, ps;
    bool stdoff;
    if (r.player == 0) {
        last = oh ? __ffs(oh) - 1 : 18;
        stdoff = last + d >= 24;
        ps = 24 - d;
    } else {
        last = oh ? 31 - __clz(oh) : 5;
        stdoff = last - d < 0;
        ps = d - 1;
    }
    if (stdoff) { mv.e0 = last; mv.n++; }
    if (ps != last && ((occ >> ps) & 1u)) {
        if (mv.e0 < 0) mv.e0 = ps; else mv.e1 = ps;
        mv.n++;
    }
    return mv;
}

// k-th set bit of m (k < popc(m))
// position of the k-th (0-based) set bit of m, -1 if m has at most k set bits:
// five narrowing steps (16 / 8 / 4 / 2 / 1 bits), no loop over k
BGX_DEV int select_bit(uint32_t m, int k) {
    int base = 0, c = __popc(m & 0xFFFFu);
    if (k >= c) { k -= c; m >>= 16; base += 16; }
    c = __popc(m & 0xFFu);
    if (k >= c) { k -= c; m >>= 8; base += 8; }
    c = __popc(m & 0xFu);
    if (k >= c) { k -= c; m >>= 4; base += 4; }
    c = __popc(m & 0x3u);
    if (k >= c) { k -= c; m >>= 2; base += 2; }
    c = (int)(m & 1u);
    if (k >= c) { k -= c; m >>= 1; base += 1; }
    return (k == 0 && (m & 1u)) ? base : -1;
}
BGX_DEV int move_source(const Moves& mv, int k) {
    if (k < mv.nsrc) return select_bit(mv.src, k);
    return k == mv.nsrc ? mv.e0 : mv.e1;
}

// apply SubMove with source s (ImmutableBoard.move_checker, immutable_board.py:183-258)
BGX_DEV Node apply_move(const Root& r, Node n, int s, int d) {
    int dst;
    if (s == 24) {
        n.x -= 1u;
        dst = r.player == 0 ? d - 1 : 24 - d;
    } else {
        uint32_t dec = 1u << ((s & 7) * 4);
        int w = s >> 3;
        n.m0 -= w == 0 ? dec : 0u;
        n.m1 -= w == 1 ? dec : 0u;
        n.m2 -= w == 2 ? dec : 0u;
        dst = r.player == 0 ? s + d : s - d;
    }
    if (dst < 0 || dst > 23) {
        n.x += 16u;  // bear off
    } else {
        uint32_t inc = 1u << ((dst & 7) * 4);
        int w = dst >> 3;
        n.m0 += w == 0 ? inc : 0u;
        n.m1 += w == 1 ? inc : 0u;
        n.m2 += w == 2 ? inc : 0u;
        uint32_t bit = 1u << dst;
        if ((r.blot & bit) && !((n.x >> 8) & bit)) n.x |= bit << 8;   // hit (check_if_blot)
    }
    return n;
}

// ------------------------------------------------------------ wave helpers
BGX_DEV int lane_id() { return (int)__lane_id(); }
BGX_DEV uint64_t ballot(bool p) { return __ballot(p); }
// number of set lanes below this lane in mask
BGX_DEV int mask_prefix(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
BGX_DEV int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
BGX_DEV uint32_t uniformu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// compiler-level ordering point for intra-wave LDS hand-offs (a wave issues
// its LDS instructions in order)
BGX_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// inclusive wave scan (64 lanes) of v
// Inclusive wave scan on DPP (row_shr within 16-lane rows, then row_bcast15 /
// row_bcast31 across rows): VALU-only, no LDS round trips.
template <int CTRL, int ROW_MASK>
BGX_DEV int dpp_add(int v) {
    return v + __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, CTRL < 0x140);
}
template <int CTRL, int ROW_MASK>
BGX_DEV int dpp_max(int v) {   // v >= 0
    const int t = __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, CTRL < 0x140);
    return v > t ? v : t;
}
BGX_DEV int wave_incl_scan(int v) {
    v = dpp_add<0x111, 0xF>(v);   // row_shr:1
    v = dpp_add<0x112, 0xF>(v);   // row_shr:2
    v = dpp_add<0x114, 0xF>(v);   // row_shr:4
    v = dpp_add<0x118, 0xF>(v);   // row_shr:8
    v = dpp_add<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
    v = dpp_add<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}
BGX_DEV int wave_incl_max(int v) {   // v >= 0
    v = dpp_max<0x111, 0xF>(v);
    v = dpp_max<0x112, 0xF>(v);
    v = dpp_max<0x114, 0xF>(v);
    v = dpp_max<0x118, 0xF>(v);
    v = dpp_max<0x142, 0xA>(v);
    v = dpp_max<0x143, 0xC>(v);
    return v;
}
BGX_DEV int lane63(int v) { return __builtin_amdgcn_readlane(v, 63); }
BGX_DEV float lane63f(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }
// float versions (DPP, VALU latency instead of ds_bpermute shuffles)
template <int CTRL, int ROW_MASK>
BGX_DEV float dpp_addf(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, CTRL < 0x140));
}
template <int CTRL, int ROW_MASK>
BGX_DEV float dpp_maxf(float v) {   // lanes without a source keep -inf
    const float t = __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
    return fmaxf(v, t);
}
BGX_DEV float wave_incl_scanf(float v) {
    v = dpp_addf<0x111, 0xF>(v);
    v = dpp_addf<0x112, 0xF>(v);
    v = dpp_addf<0x114, 0xF>(v);
    v = dpp_addf<0x118, 0xF>(v);
    v = dpp_addf<0x142, 0xA>(v);
    v = dpp_addf<0x143, 0xC>(v);
    return v;
}
BGX_DEV float wave_incl_maxf(float v) {
    v = dpp_maxf<0x111, 0xF>(v);
    v = dpp_maxf<0x112, 0xF>(v);
    v = dpp_maxf<0x114, 0xF>(v);
    v = dpp_maxf<0x118, 0xF>(v);
    v = dpp_maxf<0x142, 0xA>(v);
    v = dpp_maxf<0x143, 0xC>(v);
    return v;
}
// half-wave (lanes 32h .. 32h + 31) versions: row_shr within 16-lane rows,
// then row_bcast:15 into rows 1 and 3 (no row_bcast:31, which crosses halves)
BGX_DEV float half_incl_scanf(float v) {
    v = dpp_addf<0x111, 0xF>(v);
    v = dpp_addf<0x112, 0xF>(v);
    v = dpp_addf<0x114, 0xF>(v);
    v = dpp_addf<0x118, 0xF>(v);
    v = dpp_addf<0x142, 0xA>(v);
    return v;
}
BGX_DEV float half_incl_maxf(float v) {
    v = dpp_maxf<0x111, 0xF>(v);
    v = dpp_maxf<0x112, 0xF>(v);
    v = dpp_maxf<0x114, 0xF>(v);
    v = dpp_maxf<0x118, 0xF>(v);
    v = dpp_maxf<0x142, 0xA>(v);
    return v;
}
// the half-wave's lane 31 value (its inclusive total) to every lane of the half:
// two v_readlane (lanes 31 and 63, whatever EXEC is) and a select, no LDS
// permute round trip (the other half's value, possibly stale, is discarded)
BGX_DEV float half_last(float v) {
    const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 31));
    const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
    return (lane_id() & 32) ? b : a;
}
BGX_DEV int wave_sum(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace bgx
