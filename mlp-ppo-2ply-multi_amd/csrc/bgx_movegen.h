// bgx_movegen.h — K2 device code (move generation + afterstate expansion), shared by
// the movegen kernels (bgx_movegen.hip) and the fused 1-ply lane kernel (bgx_fused.hip).
// Algorithm notes: see the header comment of bgx_movegen.hip.
#pragma once
#include "bgx_device.h"
#include "bgx_kernels.h"

#include <cstdlib>

namespace bgx {

// Diagnostic builds only (-DBGX_STAMP, tools/stamp_build.sh): per-section
// shader-clock sums of the tier-1 job, lane 0 of each wave, per CU slot.
#ifdef BGX_STAMP
static __device__ unsigned long long bgx_stamp_acc[256 * 32];
#define STAMP_BEGIN unsigned long long stamp_last = __builtin_amdgcn_s_memtime()
#define STAMP(k)                                                                                        \
    do {                                                                                                \
        const unsigned long long stamp_c = __builtin_amdgcn_s_memtime();                                \
        if (__lane_id() == 0) atomicAdd(&bgx_stamp_acc[(blockIdx.x & 255) * 32 + (k)], stamp_c - stamp_last); \
        stamp_last = stamp_c;                                                                           \
    } while (0)
#define STAMP_COUNT(k) \
    do { if (__lane_id() == 0) atomicAdd(&bgx_stamp_acc[(blockIdx.x & 255) * 32 + (k)], 1ull); } while (0)
#else
#define STAMP_BEGIN
#define STAMP(k)
#define STAMP_COUNT(k)
#endif

// Development builds (-DBGX_DBL_GUARD=1, tools/runs/dbl_guard.sh): every global
// write of the movegen kernels, and the reply launch's input reads, check their
// index and set an error bit (0x100..0x8000, reported as "overflow flags" by the
// ABI) instead of touching memory out of range.
#ifndef BGX_DBL_GUARD
#define BGX_DBL_GUARD 0
#endif

constexpr unsigned long long EMPTY64 = ~0ull;
constexpr uint32_t KEY_EMPTY4 = 0xFFFFFu;   // four empty 5-bit fields
constexpr uint32_t KEYMASK = 0xFFFFFu;
constexpr uint32_t FLAG1 = 0x80000000u;      // "parent had exactly one move"
// LDS slices: tier 1 runs every job in SLICE_T1 bytes (512-slot table + two
// 512-entry frontiers = 8 KB, 20 waves per CU); a job whose level outgrows it
// is re-run by tier 2 in a 32 KB slice (2048 slots), and what still overflows
// by the global-memory kernel. Results are identical in every tier.
// slice = table [S] u64 | fa [S - 32] u32 | fb [S - 32] u32 | map [64] u32
template <int S> struct Slice { static constexpr int F = S - 32, bytes = S * 8 + 2 * F * 4 + 64 * 4; };
constexpr int S_T1 = 512;
constexpr int S_T2 = 2048;

struct Mem {
    unsigned long long* tab;   // [S]
    uint32_t* fa;              // [F]
    uint32_t* fb;              // [F]
    uint32_t* map;             // [64] parent start marks for one child chunk (kept zero between uses)
    int S, F;
    int force_table = 0;       // test hook (MovegenArgs::force_table): hash-table path for every job
    // lists of the table-free modes (doubles by path, non-doubles by rule); they
    // never touch the table, so a slice may lay them over it (pool kernel):
    // null = use fa / fb / F
    uint32_t* pa = nullptr;
    uint32_t* pb = nullptr;
    int PF = 0;
};

// LDS (wavefront scope) or global (agent scope) accessors
template <bool G> BGX_DEV uint32_t ld32(const uint32_t* p) {
    if constexpr (G) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV void st32(uint32_t* p, uint32_t v) {
    if constexpr (G) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV unsigned long long ld64(const unsigned long long* p) {
    if constexpr (G) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV void st64(unsigned long long* p, unsigned long long v) {
    if constexpr (G) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV unsigned long long cas64(unsigned long long* p, unsigned long long v) {
    unsigned long long cmp = EMPTY64;
    if constexpr (G)
        __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WAVEFRONT);
    return cmp;
}
template <bool G> BGX_DEV void min64(unsigned long long* p, unsigned long long v) {
    if constexpr (G) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <bool G> BGX_DEV void sync() {
    if constexpr (G) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else {
        wave_sync();
    }
}
template <bool G> BGX_DEV void clear_tab(const Mem& M) {
    for (int i = lane_id(); i < M.S; i += 64) st64<G>(M.tab + i, EMPTY64);
    sync<G>();
}

BGX_DEV uint32_t hash32(uint32_t k) {
    k ^= k >> 15;
    k *= 0x2C1B3C6Du;
    k ^= k >> 12;
    k *= 0x297A2D39u;
    return k ^ (k >> 15);
}

// Insert (key, ord) for active lanes; returns the slot holding each lane's key.
// `fresh` = this lane's CAS created the slot (a key new to the table).
template <bool G>
BGX_DEV uint32_t dedup_insert(const Mem& M, bool active, uint32_t key, uint32_t ord, bool& fresh) {
    const uint32_t mask = (uint32_t)M.S - 1u;
    uint32_t slot = hash32(key) & mask;
    const unsigned long long v = ((unsigned long long)key << 32) | ord;
    bool pending = active;
    fresh = false;
    while (ballot(pending)) {
        if (pending) {
            const unsigned long long old = cas64<G>(M.tab + slot, v);
            if (old == EMPTY64) {
                pending = false;
                fresh = true;
            } else if ((uint32_t)(old >> 32) == key) {
                if ((uint32_t)old > ord) min64<G>(M.tab + slot, v);
                pending = false;
            } else {
                slot = (slot + 1u) & mask;
            }
        }
    }
    return slot;
}

// ------------------------------------------------------------------ keys
// doubles: sorted multiset of relative step sources (0 = BAR, then travel order)
BGX_DEV uint32_t rel_of(int s, int player) {
    if (s == 24) return 0u;
    return player == 0 ? (uint32_t)(s + 1) : (uint32_t)(24 - s);
}
BGX_DEV int abs_of(uint32_t rel, int player) {
    if (rel == 0u) return 24;
    return player == 0 ? (int)rel - 1 : 24 - (int)rel;
}
BGX_DEV uint32_t key_insert(uint32_t key, uint32_t rel) {
    uint32_t out = 0;
    int o = 0;
    bool placed = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t f = (key >> (5 * i)) & 31u;
        if (!placed && rel <= f) { out |= rel << (5 * o); ++o; placed = true; }
        if (o < 4) { out |= f << (5 * o); ++o; }
    }
    return out;
}
BGX_DEV Node rebuild(const Root& R, uint32_t key, int d) {
    Node n = root_node(R);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t f = (key >> (5 * i)) & 31u;
        if (f != 31u) n = apply_move(R, n, abs_of(f, R.player), d);
    }
    return n;
}

// ---- doubles without a table (first-reach paths only) ----------------------
// Outside bear-off a node's move list is its movable sources in ascending
// position (bar entry alone while on the bar), so the first-reach path of a
// board (the lexicographically smallest index sequence, which the reference's
// DFS records) takes, at every step, the lowest source movable there. A path
// is first-reach iff no later step uses a source that was movable, and lower,
// at an earlier step. Keeping only such paths gives every board once, already
// in first-reach order: no hash table, no dedup, no duplicate children.
// Valid when no node of the tree can be in bear-off (>= 5 mover checkers
// outside home, bar included); other jobs take the table path.
constexpr uint32_t PATHF = 0x40000000u;        // frontier / record entry is a path
constexpr uint32_t PATH_EMPTY = KEY_EMPTY4;   // four empty 5-bit fields

BGX_DEV bool doubles_by_path(const Root& R) {
    const uint32_t home = R.player == 0 ? nibsum(R.m2 >> 8) : nibsum(R.m0 & 0xFFFFFFu);
    return 15u - R.off - home >= 5u;   // outside home (points and bar)
}
// The state after a path's steps (abs sources, in order) that the moves and
// the first-reach filter need -- the mover's occupancy (kept up to date per
// step: the source empties when it held one checker, the destination fills),
// its bar count (returned) and the sources the path rules out (movable at an
// earlier step and below that step's source) -- without building the board:
// a source's count before a step is its root count plus the earlier steps
// that landed on it minus those that left it. (path_board builds the board of
// a record.)
BGX_DEV uint32_t path_state(const Root& R, uint32_t path, int d, uint32_t okd, uint32_t& bad, uint32_t& occ) {
    bad = 0u;
    occ = occ24(R.m0, R.m1, R.m2);
    uint32_t bar = R.bar;
    int src[4], dst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t f = (path >> (5 * i)) & 31u;
        src[i] = -1;
        dst[i] = -1;
        if (f != 31u) {
            int t;
            if (f < 24u) {
                bad |= occ & okd & ((1u << f) - 1u);
                int c = (int)nib(R.m0, R.m1, R.m2, (int)f);
#pragma unroll
                for (int j = 0; j < i; ++j) c += (dst[j] == (int)f ? 1 : 0) - (src[j] == (int)f ? 1 : 0);
                if (c == 1) occ &= ~(1u << f);
                t = R.player == 0 ? (int)f + d : (int)f - d;
            } else {
                bar -= 1u;
                t = R.player == 0 ? d - 1 : 24 - d;
            }
            src[i] = (int)f;
            dst[i] = t;
            if (t >= 0 && t <= 23) occ |= 1u << t;
        }
    }
    return bar;
}
// a node's move list in a path-mode job (no node of its tree can be in
// bear-off: doubles_by_path): the bar entry while on the bar, else every
// occupied point whose destination is open (get_moves_bar / get_moves_normal,
// get_moves_one_die.py:40-130) -- node_moves without the bear-off analysis
BGX_DEV Moves path_moves(const Root& R, uint32_t bar, uint32_t occ, int d, uint32_t okd) {
    Moves mv;
    mv.src = 0; mv.nsrc = 0; mv.e0 = -1; mv.e1 = -1; mv.n = 0;
    if (bar > 0u) {
        const int entry = R.player == 0 ? d - 1 : 24 - d;
        if (!((R.block >> entry) & 1u)) { mv.e0 = 24; mv.n = 1; }
        return mv;
    }
    mv.src = occ & okd;
    mv.nsrc = __popc(mv.src);
    mv.n = mv.nsrc;
    return mv;
}
BGX_DEV Node path_board(const Root& R, uint32_t path, int d) {
    Node n = root_node(R);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t f = (path >> (5 * i)) & 31u;
        if (f != 31u) n = apply_move(R, n, (int)f, d);
    }
    return n;
}

// non-doubles: positions 0..23 points, 24 = BAR (source), 25 = OFF (dest), 31 = none
BGX_DEV int dest_of(const Root& R, int s, int d) {
    const int t = s == 24 ? (R.player == 0 ? d - 1 : 24 - d) : (R.player == 0 ? s + d : s - d);
    return (t < 0 || t > 23) ? 25 : t;
}
BGX_DEV uint32_t sort2(uint32_t a, uint32_t b) { return a <= b ? (a | (b << 5)) : (b | (a << 5)); }
// canonical key of the board after steps (s1->t1, hit h1) and (s2->t2, hit h2); s2 = 31: single
BGX_DEV uint32_t nd_key(uint32_t s1, uint32_t t1, bool h1, uint32_t s2, uint32_t t2, bool h2) {
    uint32_t r0 = s1, r1 = s2, a0 = t1, a1 = t2;
    if (s2 != 31u) {
        if (t1 == s2) { r1 = 31u; a0 = 31u; }        // chained checker: s1 -> t1 -> t2
        else if (t2 == s1) { r0 = 31u; a1 = 31u; }   // s2 -> s1 -> t1
    }
    const uint32_t hh0 = h1 ? t1 : 31u, hh1 = h2 ? t2 : 31u;
    return sort2(r0, r1) | (sort2(a0, a1) << 10) | (sort2(hh0, hh1) << 20);
}

// Non-doubles without a table. With nothing on the bar and >= 3 mover
// checkers outside home no node of the two-step tree is in bear-off, and the
// 2-move plays enumerated in (pass, i, j) order (pass 0: high die first) fall
// into two kinds:
//  - two checkers (no step lands on the other's source): the pass-0 play
//    (a with H, b with L) is the only pass-0 producer of its board and its
//    pass-1 twin (b with L, a with H) is always legal: keep pass 0 only;
//  - one checker x moving H + L: producers A = pass-0 chain x -> x+H -> .,
//    B = pass-0 reverse (x+L with H, then x with L; x+L mover-occupied),
//    C = pass-1 chain x -> x+L -> ., D = pass-1 reverse (x+H with L, then x
//    with H). A chain that hits at its intermediate point makes a board no
//    other play makes; the others make the same board and the first legal one
//    in enumeration order (ascending first source within a pass) is kept.
// This reproduces first-occurrence dedup (handle_non_doubles,
// generate_all_moves.py:28-68) exactly on those positions; others use the table.
constexpr uint32_t ND_DROP = 0xFFFFFFFFu;
BGX_DEV bool nd_by_rule(const Root& R) {
    const uint32_t home = R.player == 0 ? nibsum(R.m2 >> 8) : nibsum(R.m0 & 0xFFFFFFu);
    return R.bar == 0u && 15u - R.off - home >= 3u;
}
BGX_DEV bool nd_first(const Root& R, uint32_t occ0, int pass, int s1, int t1, int s2, int t2, int H, int L) {
    const bool chain = s2 == t1;
    if (!chain && t2 != s1) return pass == 0;
    if (chain && ((R.blot >> t1) & 1u)) return true;
    const int x = chain ? s1 : s2;
    const int iH = R.player == 0 ? x + H : x - H, iL = R.player == 0 ? x + L : x - L;
    const uint32_t bad = R.block | R.blot;
    const bool A = !((bad >> iH) & 1u), B = (occ0 >> iL) & 1u;
    const bool C = !((bad >> iL) & 1u), D = (occ0 >> iH) & 1u;
    // rank in enumeration order: player 0 (sources ascend with travel) A B C D,
    // player 1 B A D C
    const int me = pass == 0 ? (chain ? 0 : 1) : (chain ? 2 : 3);
    const bool p0 = R.player == 0;
    switch (me) {
        case 0: return p0 ? true : !B;
        case 1: return p0 ? !A : true;
        case 2: return !A && !B && (p0 ? true : !D);
        default: return !A && !B && (p0 ? !C : true);
    }
}
BGX_DEV void nib_add(Node& n, int p, int delta) {
    const uint32_t v = 1u << ((p & 7) * 4);
    const int w = p >> 3;
    if (delta > 0) {
        n.m0 += w == 0 ? v : 0u; n.m1 += w == 1 ? v : 0u; n.m2 += w == 2 ? v : 0u;
    } else {
        n.m0 -= w == 0 ? v : 0u; n.m1 -= w == 1 ? v : 0u; n.m2 -= w == 2 ? v : 0u;
    }
}
BGX_DEV Node nd_board(const Root& R, uint32_t key) {
    Node n = root_node(R);
    // additions first, so a removal never borrows from a neighbouring nibble
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t a = (key >> (10 + 5 * i)) & 31u, h = (key >> (20 + 5 * i)) & 31u;
        if (a == 25u) n.x += 16u;
        else if (a < 24u) nib_add(n, (int)a, +1);
        if (h < 24u) n.x |= 1u << (8 + h);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t r = (key >> (5 * i)) & 31u;
        if (r == 24u) n.x -= 1u;
        else if (r < 24u) nib_add(n, (int)r, -1);
    }
    return n;
}

// ------------------------------------------------------------------ job I/O
struct JobIn { Root R; int d0, d1; bool skip; };
BGX_DEV JobIn make_job(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4, uint32_t w5, uint32_t w6,
                       int player, int d0, int d1);

// A job's input as loaded (fetch_raw), before the root analysis (decode_job):
// the split lets a kernel load the next job's words while the current one runs.
// One register per lane: lane k < 8 holds word k of the packed board (lane
// k < 13: word k of the u8[52] board in IN_U8 mode), lane 13 the mover and dice
// (player | d0 << 8 | d1 << 16; not IN_TWOPLY, where they follow from the row
// and the job index); decode_job reads them back with readlane (SGPRs).
// IN_TWOPLY rows whose word 7 is SKIP_ROW are skipped (a lane with fewer than
// four candidates, two_ply.py:67-70 via the engine's top-k).
constexpr uint32_t SKIP_ROW = 0xFFFFFFFFu;
struct RawJob { uint32_t v; };

BGX_DEV int job_count(const MovegenArgs& a) {
    int n = a.n_jobs;
    if (a.n_jobs_dev) n += (int)(*a.n_jobs_dev) * a.jobs_per_dev_unit;
    if (a.n_jobs_max > 0 && n > a.n_jobs_max) n = a.n_jobs_max;
    return n;
}


BGX_DEV RawJob fetch_raw(const MovegenArgs& a, int j) {
    const int l = lane_id();
    uint32_t v = 0u;
    if (a.in_mode == IN_U8) {
        if (l < 13) v = ((const uint32_t*)(a.in_u8 + (size_t)j * 52))[l];
    } else {
        int src = j;
        if (a.in_mode == IN_TWOPLY) {
            const int row = j / 21;
            if (BGX_DBL_GUARD && (j < 0 || j >= job_count(a))) {
                if (l == 0) atomicOr(a.err_flags, 0x8000u);
                return {0u};
            }
            src = a.in_rows ? a.in_rows[row] : a.in_row_base + row;
        }
        if (l < 8) v = src < 0 ? (l == 7 ? SKIP_ROW : 0u) : a.in_packed[(size_t)src * 8 + l];
    }
    if (l == 13 && a.in_mode != IN_TWOPLY)
        v = (uint32_t)a.in_player[j] | ((uint32_t)a.in_dice[2 * j] << 8) | ((uint32_t)a.in_dice[2 * j + 1] << 16);
    return {v};
}

BGX_DEV uint32_t lane_word(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }

BGX_DEV JobIn decode_job(const MovegenArgs& a, int j, const RawJob& r) {
    uint32_t w[7];
    if (a.in_mode == IN_U8) {
#pragma unroll
        for (int k = 0; k < 6; ++k) w[k] = pack4(lane_word(r.v, 2 * k)) | (pack4(lane_word(r.v, 2 * k + 1)) << 16);
        const uint32_t t = lane_word(r.v, 12);
        w[6] = (t & 15u) | (((t >> 8) & 15u) << 4) | (((t >> 16) & 15u) << 8) | (((t >> 24) & 15u) << 12);
    } else {
#pragma unroll
        for (int k = 0; k < 7; ++k) w[k] = lane_word(r.v, k);
    }
    const uint32_t pd = lane_word(r.v, 13);
    int player = (int)(pd & 255u), d0 = (int)((pd >> 8) & 255u), d1 = (int)(pd >> 16);
    bool skip = false;
    if (a.in_mode == IN_TWOPLY) {
        skip = lane_word(r.v, 7) == SKIP_ROW;
        // two_ply.py:93-150: the opponent of the candidate's mover replies to every roll
        player = 1 - (int)((w[6] >> 16) & 1u);
        int a0 = 1, q = j - 21 * (j / 21);   // DICE_ROLLS order (two_ply.py:10-32)
        while (q >= 7 - a0) { q -= 7 - a0; ++a0; }
        d0 = a0;
        d1 = a0 + q;
    }
    JobIn in = make_job(w[0], w[1], w[2], w[3], w[4], w[5], w[6], player, d0, d1);
    in.skip = skip;
    return in;
}

BGX_DEV JobIn fetch_job(const MovegenArgs& a, int j) { return decode_job(a, j, fetch_raw(a, j)); }

// job from a packed board's words 0..6, the mover and the dice
BGX_DEV JobIn make_job(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4, uint32_t w5, uint32_t w6,
                       int player, int d0, int d1) {
    JobIn in;
    in.skip = false;
    // the job is wave-uniform: pin its words in SGPRs so the root analysis
    // below (and node_moves on the root) runs on the scalar unit, not VALU
    w0 = uniformu(w0); w1 = uniformu(w1); w2 = uniformu(w2); w3 = uniformu(w3);
    w4 = uniformu(w4); w5 = uniformu(w5); w6 = uniformu(w6);
    player = uniform(player);
    in.d0 = uniform(d0);
    in.d1 = uniform(d1);
    const bool p2 = player != 0;
    Root& R = in.R;
    R.m0 = p2 ? w3 : w0; R.m1 = p2 ? w4 : w1; R.m2 = p2 ? w5 : w2;
    R.o0 = p2 ? w0 : w3; R.o1 = p2 ? w1 : w4; R.o2 = p2 ? w2 : w5;
    const uint32_t b0 = w6 & 15u, b1 = (w6 >> 4) & 15u, f0 = (w6 >> 8) & 15u, f1 = (w6 >> 12) & 15u;
    R.bar = p2 ? b1 : b0; R.obar = p2 ? b0 : b1;
    R.off = p2 ? f1 : f0; R.ooff = p2 ? f0 : f1;
    R.block = ge2_24(R.o0, R.o1, R.o2);
    R.blot = occ24(R.o0, R.o1, R.o2) & ~R.block;
    R.player = player;
    return in;
}

// write record k of job j (lane-local)
BGX_DEV void emit_one(const MovegenArgs& a, int j, const Root& R, const Node& n, int k, int base) {
    uint32_t w[8];
    node_to_packed(R, n, (uint32_t)R.player, w);
    if (a.out_mode == OUT_U8) {
        if (k >= a.cap) return;
        uint32_t o[13];
        packed_to_u8(w, o);
        uint32_t* dst = (uint32_t*)(a.out_u8 + ((size_t)j * a.cap + k) * 52);
#pragma unroll
        for (int i = 0; i < 13; ++i) dst[i] = o[i];
        return;
    }
    size_t row;
    if (a.out_mode == OUT_PACKED_SLOT) {
        if (k >= a.cap) return;
        row = (size_t)j * a.cap + k;
    } else {
        if (BGX_DBL_GUARD && (base < 0 || k < 0 || base + k >= a.flat_cap)) {
            atomicOr(a.err_flags, 0x2000u);
            return;
        }
        row = (size_t)base + k;
    }
    // a 2-ply reply row carries its root slot (the candidate it answers: job / 21)
    // in word 7, so the reply MLP can evaluate it by difference from the root
    // (mlp_kernel_delta, bgx_mlp.hip)
    if (a.in_mode == IN_TWOPLY) w[7] = (uint32_t)j / 21u;
    uint4* dst = (uint4*)(a.out_packed + row * 8);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// Per-wave output reservation for OUT_PACKED_FLAT: one global atomic per
// `flat_chunk` rows instead of one per job (a single counter hit by every job
// of a 2-ply launch serialises at the memory side).
// left_hint >= 0: the jobs this wave still expects (kernels that do not
// stride by gridDim.x set it per job; begin_emit sizes its reservation by it)
// (base2, left2): the larger remainder of an earlier chunk, kept when a request
// did not fit it (a 2-ply row block of ~200 rows would otherwise leave up to a
// block's worth of gap rows per chunk, which the reply MLP evaluates)
// wg (the reply launch): requests that neither remainder holds are served from
// a workgroup-level chunk in LDS (WgRows) instead of a global atomic per wave
// chunk; a wave's unused chunk tail at the end of the launch was a gap row
// block of up to flat_chunk rows per wave (14 % of a K = 4 launch's rows, 7 %
// at K = all), while the workgroup sizes its chunks by its remaining items and
// leaves one small tail per workgroup.
struct WgRows {
    unsigned long long span;   // current chunk: next free row (low 32 bits), end (high 32)
    unsigned used;             // rows handed to requests so far
    int next, done, items;     // the workgroup's items: claimed (its LDS item counter), finished, all
};
struct FlatCursor {
    int base = 0, left = 0, left_hint = -1, base2 = 0, left2 = 0;
    WgRows* wg = nullptr;   // LDS, or null: per-wave chunks from the global counter
};

// n rows from the cursor's current or kept remainder; false: neither holds them
BGX_DEV bool cursor_take(FlatCursor& fc, int n, int& base) {
    if (n <= fc.left) {
        base = fc.base;
        fc.base += n;
        fc.left -= n;
        return true;
    }
    if (n <= fc.left2) {
        base = fc.base2;
        fc.base2 += n;
        fc.left2 -= n;
        return true;
    }
    return false;
}
// a new chunk replaces the current one; the larger of the two remainders is kept
BGX_DEV void cursor_new_chunk(FlatCursor& fc, int base, int n, int grab) {
    if (fc.left > fc.left2) {
        fc.base2 = fc.base;
        fc.left2 = fc.left;
    }
    fc.base = base + n;
    fc.left = grab - n;
}

// n rows from the workgroup's chunk (lane 0 decides, the result is broadcast);
// -1: the flat buffer is full (flagged). A request the chunk cannot hold
// locks the span (bit 31 of its end), refills it with a global reservation
// sized by the workgroup's progress -- rows per item so far x (items not yet
// claimed + a quarter of the items in flight), between max(n, 64) and 8 x flat_chunk,
// so the chunks shrink as the workgroup's items run out -- and unlocks it;
// requests that meet the lock wait for the new chunk (one refill at a time:
// concurrent refills each kept a chunk, 16 per workgroup at a launch's start).
// The replaced chunk's tail becomes the refilling wave's own remainder.
constexpr unsigned WG_LOCK = 0x80000000u;
BGX_DEV int wg_take(const MovegenArgs& a, int n, FlatCursor& fc) {
    int b = 0, rb = 0, rl = 0;
    if (lane_id() == 0) {
        WgRows* g = fc.wg;
        unsigned long long s = __hip_atomic_load(&g->span, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (unsigned spin = 0;;) {
            const unsigned nx = (unsigned)s, en = (unsigned)(s >> 32);
            if (en & WG_LOCK) {   // another wave is refilling
                if (++spin >= (1u << 24)) {   // bounded
                    atomicOr(a.err_flags, BGX_ERRF_WAIT_BOUND);
                    b = -1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                s = __hip_atomic_load(&g->span, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                continue;
            }
            if (nx + (unsigned)n <= en) {
                const unsigned long long prev = atomicCAS(&g->span, s, ((unsigned long long)en << 32) | (nx + n));
                if (prev == s) {
                    b = (int)nx;
                    break;
                }
                s = prev;
                continue;
            }
            const unsigned long long lk = ((unsigned long long)(en | WG_LOCK) << 32) | nx;
            const unsigned long long prev = atomicCAS(&g->span, s, lk);
            if (prev != s) {
                s = prev;
                continue;
            }
            const int items = g->items;
            int claimed = __hip_atomic_load(&g->next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (claimed > items) claimed = items;
            const int done = __hip_atomic_load(&g->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int flight = claimed > done ? claimed - done : 0;
            const unsigned used = __hip_atomic_load(&g->used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            // prior: ~107 records per item at K = 4 (8,192 lanes, 12/64 per-roll tail)
            const float per_item = used ? (float)used / (float)(2 * done + flight + 1) * 2.0f : 128.0f;
            const int cap = 8 * a.flat_chunk;
            const float want_f = per_item * ((float)(items - claimed) + 0.25f * (float)flight + 0.5f);
            int want = want_f > (float)cap ? cap : (int)want_f;
            if (want < 64) want = 64;
            const int grab = n > want ? n : want;
            const int gb = (int)atomicAdd(a.flat_count, (unsigned)grab);
            if (gb + grab > a.flat_cap) {
                atomicOr(a.err_flags, BGX_ERRF_FLAT_OVERFLOW);
                __hip_atomic_store(&g->span, ((unsigned long long)en << 32) | en, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                b = -1;
                break;
            }
            __hip_atomic_store(&g->span, ((unsigned long long)(unsigned)(gb + grab) << 32) | (unsigned)(gb + n),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            b = gb;
            rb = (int)nx;   // the replaced chunk's tail: this wave's now
            rl = (int)(en - nx);
            break;
        }
        if (b >= 0) atomicAdd(&g->used, (unsigned)n);
    }
    b = uniform(b);
    rb = uniform(rb);
    rl = uniform(rl);
    if (b < 0) {
        fc.left = fc.left2 = 0;
        return -1;
    }
    // keep the larger two of (current, kept, new) remainders
    if (rl > fc.left) {
        if (fc.left > fc.left2) {
            fc.base2 = fc.base;
            fc.left2 = fc.left;
        }
        fc.base = rb;
        fc.left = rl;
    } else if (rl > fc.left2) {
        fc.base2 = rb;
        fc.left2 = rl;
    }
    return b;
}

// reserve output space once the job's record count is known; returns base (-1: overflow)
BGX_DEV int begin_emit(const MovegenArgs& a, int j, int n, FlatCursor& fc) {
    int base = 0;
    if (a.out_mode == OUT_PACKED_FLAT) {
        if (cursor_take(fc, n, base)) {
        } else if (fc.wg) {
            base = wg_take(a, n, fc);
        } else {
            // chunk = min(flat_chunk, 32 rows per job this wave still has), at least n
            const int left_jobs =
                fc.left_hint >= 0 ? fc.left_hint : (job_count(a) - j + (int)gridDim.x - 1) / (int)gridDim.x;
            int want = 32 * left_jobs;
            if (want > a.flat_chunk) want = a.flat_chunk;
            const int grab = n > want ? n : want;
            if (lane_id() == 0) base = (int)atomicAdd(a.flat_count, (unsigned)grab);
            base = uniform(base);
            if (base + grab > a.flat_cap) {
                if (lane_id() == 0) atomicOr(a.err_flags, BGX_ERRF_FLAT_OVERFLOW);
                fc.left = fc.left2 = 0;
                base = -1;
            } else {
                cursor_new_chunk(fc, base, n, grab);
            }
        }
        if (lane_id() == 0) {
            if (BGX_DBL_GUARD && (j < 0 || j >= job_count(a))) {
                atomicOr(a.err_flags, 0x1000u);
            } else {
                a.job_off[j] = base < 0 ? 0 : base;
                a.job_cnt[j] = base < 0 ? 0 : n;
            }
        }
    } else if (lane_id() == 0) {
        a.out_count[j] = n;
    }
    return base;
}

// ------------------------------------------------------------------ expansion
// j-th set bit (0-based) of a 24-bit mask, j < popcount(m): branch-free narrowing
BGX_DEV int select_bit_fast(uint32_t m, int j) {
    int base = 0;
    int c = __popc(m & 0xFFFu);
    if (j >= c) { j -= c; m >>= 12; base += 12; }
    c = __popc(m & 0x3Fu);
    if (j >= c) { j -= c; m >>= 6; base += 6; }
    c = __popc(m & 0x7u);
    if (j >= c) { j -= c; m >>= 3; base += 3; }
    m = j >= 1 ? (m & (m - 1u)) : m;
    m = j >= 2 ? (m & (m - 1u)) : m;
    return base + __ffs(m) - 1;
}

// would appending T entries at n overflow a list of F?
BGX_DEV bool n_out_check(int n, int T, int F) { return n + T > F; }

// Parent lane of child r = b + lane in a flat enumeration: the last lane q
// with c > 0 and excl <= r. Parents starting inside [b, b + 64) mark
// map[excl - b] = q + 1; a max-scan over the marks fills the gaps; before the
// first mark it is q0. `map` (64 words) is zero on entry and on return.
template <bool G>
BGX_DEV int flat_parent(uint32_t* map, int excl, int c, int b) {
    const int l = lane_id();
    const int st = excl - b;
    if (c > 0 && st >= 0 && st < 64) st32<G>(map + st, (uint32_t)(l + 1));
    const uint64_t cov = ballot(c > 0 && excl <= b);
    const int q0 = cov ? 63 - __clzll((long long)cov) : 0;
    sync<G>();
    const int mk = wave_incl_max((int)ld32<G>(map + l));
    st32<G>(map + l, 0u);
    return mk ? mk - 1 : q0;
}

// Expand one chunk of parents (one per lane, c = its move count, c = 0 for
// none). Children are enumerated FLAT in (parent, move) = ordinal order, one
// per lane: the parent is the largest lane p with exclusive-prefix <= r (six
// shuffle steps), its move list comes over by shuffles, kfn(p, s) gives the
// child's key. Each 64-child chunk is deduplicated in one round; survivors
// (first occurrences) are appended to `out` in order with payload key | tag.
// Returns false when the table or the list would overflow (fallback path).
template <bool G, typename KeyFn>
BGX_DEV bool expand_flat(const Mem& M, const Moves& pm, int c, uint32_t tagbit, uint32_t ord_base, KeyFn kfn,
                         uint32_t* out, int& n_out, int& inserted, uint32_t& total) {
    const int l = lane_id();
    const int incl = wave_incl_scan(c);
    const int excl = incl - c;
    const int T = lane63(incl);
    total = (uint32_t)T;
    for (int b = 0; b < T; b += 64) {
        const int r = b + l;
        const bool act = r < T;
        const int p = flat_parent<G>(M.map, excl, c, b);
        const int j = r - __shfl(excl, p, 64);
        const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
        const int nsrc = __shfl(pm.nsrc, p, 64);
        const int e0 = __shfl(pm.e0, p, 64), e1 = __shfl(pm.e1, p, 64);
        const uint32_t tag = (uint32_t)__shfl((int)tagbit, p, 64);
        const int s = j < nsrc ? select_bit_fast(src, j) : (j == nsrc ? e0 : e1);
        const uint32_t key = kfn(p, s);
        const uint32_t ord = ord_base + (uint32_t)r;
        bool fresh;
        const uint32_t slot = dedup_insert<G>(M, act, key, ord, fresh);
        inserted += __popcll(ballot(fresh));
        if (inserted > M.S - (M.S >> 2)) {
            STAMP_COUNT(20);   // (diagnostic builds: overflow cause)
            return false;
        }
        sync<G>();
        const bool sv = act && (uint32_t)ld64<G>(M.tab + slot) == ord;
        const uint64_t bm = ballot(sv);
        // exact: the survivors of this chunk must fit the list
        if (n_out + __popcll(bm) > M.F) {
            STAMP_COUNT(21);
            return false;
        }
        if (sv) st32<G>(out + n_out + mask_prefix(bm), key | tag);
        n_out += __popcll(bm);
    }
    sync<G>();
    return true;
}

// expand_flat without a table: kfn returns ND_DROP for children that an
// earlier child already produced (nd_first); the rest are appended in order
template <bool G, typename KeyFn>
BGX_DEV bool expand_keep(const Mem& M, const Moves& pm, int c, KeyFn kfn, uint32_t* out, int& n_out, int cap) {
    const int l = lane_id();
    const int incl = wave_incl_scan(c);
    const int excl = incl - c;
    const int T = lane63(incl);
    for (int b = 0; b < T; b += 64) {
        const int r = b + l;
        const int p = flat_parent<G>(M.map, excl, c, b);
        const int j = r - __shfl(excl, p, 64);
        const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
        // kfn shuffles from the parent lane: every lane runs it (a lane
        // masked off by a branch returns nothing to ds_bpermute)
        const uint32_t key = kfn(p, select_bit_fast(src, j));
        const bool sv = r < T && key != ND_DROP;
        const uint64_t bm = ballot(sv);
        if (n_out + 64 > cap) return false;
        if (sv) st32<G>(out + n_out + mask_prefix(bm), key);
        n_out += __popcll(bm);
    }
    sync<G>();
    return true;
}

// ------------------------------------------------------------------ the job
// returns the record count, or -1 when the slice overflowed (fallback)
// heavy_t: a doubles level with more children than this returns -2 (the
// small-launch kernel then expands the job with the whole block)
template <bool G>
BGX_DEV int job_records(const JobIn& in, const Mem& M, uint32_t*& fin_out, int heavy_t) {
    STAMP_BEGIN;
    const Root& R = in.R;
    const int l = lane_id();
    const Node root = root_node(R);
    int inserted = 0;
    uint32_t* fin = M.fa;   // final record list
    int nfin = 0;
    // the table-free lists (may overlay the table)
    uint32_t* const pa = M.pa ? M.pa : M.fa;
    uint32_t* const pb = M.pa ? M.pb : M.fb;
    const int PFc = M.pa ? M.PF : M.F;
    const bool dbl = in.d0 == in.d1;
    const int d = in.d0;

    if (!dbl) {
        // ------------------------------------------------ non-doubles
        const int H = in.d0 > in.d1 ? in.d0 : in.d1, L = in.d0 > in.d1 ? in.d1 : in.d0;
        const uint32_t okH = ok_mask(R.block, H, R.player), okL = ok_mask(R.block, L, R.player);
        const Moves mH = node_moves(R, root, H, okH), mL = node_moves(R, root, L, okL);
        const int pass = (l >> 4) & 1, k = l & 15;
        const bool in32 = l < 32;
        const int dA = pass ? L : H, dB = pass ? H : L;
        const bool v1 = in32 && k < (pass ? mL.n : mH.n);
        Moves mA;
        mA.src = pass ? mL.src : mH.src;
        mA.nsrc = pass ? mL.nsrc : mH.nsrc;
        mA.e0 = pass ? mL.e0 : mH.e0;
        mA.e1 = pass ? mL.e1 : mH.e1;
        mA.n = pass ? mL.n : mH.n;
        int s1 = 0;
        if (v1) s1 = k < mA.nsrc ? select_bit_fast(mA.src, k) : (k == mA.nsrc ? mA.e0 : mA.e1);
        const uint32_t t1 = (uint32_t)dest_of(R, s1, dA);
        // rule mode (nd_by_rule: nothing on the bar, >= 3 mover checkers outside
        // home): no node of the two-step tree is on the bar or bearing off, so
        // the child's move list is its occupancy (the source empties when it
        // held one checker, t1 fills) with an open destination for dB
        const bool rule = nd_by_rule(R) && !M.force_table;
        Moves m2;
        if (rule) {
            const uint32_t last1 = nib(R.m0, R.m1, R.m2, s1) == 1u ? 1u << s1 : 0u;
            m2.src = ((occ24(R.m0, R.m1, R.m2) & ~last1) | (1u << (t1 & 31u))) & (pass ? okH : okL);
            m2.nsrc = m2.n = __popc(m2.src);
            m2.e0 = m2.e1 = -1;
        } else {
            const Node child = v1 ? apply_move(R, root, s1, dA) : root;
            m2 = node_moves(R, child, dB, pass ? okH : okL);
        }
        const int c = v1 ? m2.n : 0;
        const bool two1 = ballot(in32 && pass == 0 && c > 0) != 0ull;
        const bool two2 = ballot(in32 && pass == 1 && c > 0) != 0ull;
        const int nH = mH.n, nL = mL.n;
        const bool h1 = v1 && t1 < 24u && ((R.blot >> t1) & 1u);
        if ((two1 || (nH != 1 && two2)) && rule) {
            STAMP(1);
            STAMP_COUNT(4);
            // 2-move records without a table (nd_first): a pass-2 parent can
            // only add its chain (s2 = t1) or reverse chain (s2 -> s1) child
            if (pass == 1) {
                const int rv = R.player == 0 ? s1 - H : s1 + H;
                const uint32_t cand = (t1 < 24u ? 1u << t1 : 0u) | ((rv >= 0 && rv < 24) ? 1u << rv : 0u);
                m2.src &= cand;
                m2.nsrc = m2.n = __popc(m2.src);
            }
            const int cc = v1 ? m2.n : 0;
            const uint32_t blot2 = R.blot & ~(h1 ? (1u << t1) : 0u);
            const uint32_t occ0 = occ24(R.m0, R.m1, R.m2);
            auto kfn = [&](int p, int s2) -> uint32_t {
                const int ps1 = __shfl(s1, p, 64);
                const int pt1 = __shfl((int)t1, p, 64);
                const uint32_t pb2 = (uint32_t)__shfl((int)blot2, p, 64);
                const bool ph1 = __shfl((int)h1, p, 64) != 0;
                const int pp = p >> 4;
                const int t2 = dest_of(R, s2, pp ? H : L);
                const bool h2 = ((pb2 >> t2) & 1u) != 0u;
                const uint32_t key = nd_key((uint32_t)ps1, (uint32_t)pt1, ph1, (uint32_t)s2, (uint32_t)t2, h2);
                return nd_first(R, occ0, pp, ps1, pt1, s2, t2, H, L) ? key : ND_DROP;
            };
            fin = pa;
            if (!expand_keep<G>(M, m2, cc, kfn, fin, nfin, PFc)) {
                STAMP_COUNT(22);
                return -1;
            }
            STAMP(2);
        } else if (two1 || (nH != 1 && two2)) {
            // 2-move records in (pass, i, j) order (handle_non_doubles 43-68, both passes)
            clear_tab<G>(M);
            const int cc = in32 ? c : 0;
            const uint32_t blot2 = R.blot & ~(h1 ? (1u << t1) : 0u);
            auto kfn = [&](int p, int s2) -> uint32_t {
                const uint32_t ps1 = (uint32_t)__shfl(s1, p, 64);
                const uint32_t pt1 = (uint32_t)__shfl((int)t1, p, 64);
                const uint32_t pb2 = (uint32_t)__shfl((int)blot2, p, 64);
                const bool ph1 = __shfl((int)h1, p, 64) != 0;
                const int pdB = (p >> 4) ? H : L;
                const uint32_t t2 = (uint32_t)dest_of(R, s2, pdB);
                const bool h2 = t2 < 24u && ((pb2 >> t2) & 1u);
                return nd_key(ps1, pt1, ph1, (uint32_t)s2, t2, h2);
            };
            uint32_t tot;
            if (!expand_flat<G>(M, m2, cc, 0u, 0u, kfn, fin, nfin, inserted, tot)) {
                STAMP_COUNT(24);
                return -1;
            }
        } else {
            // singles: high-die singles, then (unless pass 2 is skipped) low-die singles
            // (handle_non_doubles 70-81; generate_all_moves.py:40-50)
            clear_tab<G>(M);
            const int nL2 = (nH == 1) ? 0 : nL;
            const bool act = v1 && (pass == 0 || k < nL2);
            const uint32_t ord = pass == 0 ? (uint32_t)k : (uint32_t)(nH + k);
            const uint32_t key = nd_key((uint32_t)s1, t1, h1, 31u, 31u, false);
            bool fresh;
            const uint32_t slot = dedup_insert<G>(M, act, key, ord, fresh);
            sync<G>();
            const bool sv = act && (uint32_t)ld64<G>(M.tab + slot) == ord;
            const uint64_t bm = ballot(sv);
            if (sv) st32<G>(fin + mask_prefix(bm), key);
            nfin = __popcll(bm);
            sync<G>();
        }
    } else {
        // ------------------------------------------------ doubles
        const uint32_t okd = ok_mask(R.block, d, R.player);
        uint32_t* fa = M.fa;
        uint32_t* fb = M.fb;
        if (doubles_by_path(R) && !M.force_table) {
            STAMP_COUNT(11);
            fa = pa;
            fb = pb;
            if (l == 0) st32<G>(fa, PATH_EMPTY);
            sync<G>();
            int n = 1, level = 0;
            while (level < 4) {
                int nn = 0;
                uint32_t T = 0;
                for (int b = 0; b < n; b += 64) {
                    const int i = b + l;
                    const bool live = i < n;
                    const uint32_t path = live ? ld32<G>(fa + i) & KEYMASK : PATH_EMPTY;
                    uint32_t bad, occ;
                    const uint32_t nbar = path_state(R, path, d, okd, bad, occ);
                    Moves pm = path_moves(R, nbar, occ, d, okd);
                    const uint32_t one = pm.n == 1 ? FLAG1 : 0u;
                    pm.src &= ~bad;                      // e0 is the bar entry (or none) here
                    pm.nsrc = __popc(pm.src);
                    const int c = live ? pm.nsrc + (pm.e0 >= 0 ? 1 : 0) : 0;
                    const int incl = wave_incl_scan(c);
                    const int excl = incl - c;
                    const int Tc = lane63(incl);
                    if (n_out_check(nn, Tc, PFc)) {
                        STAMP_COUNT(23);
                        return -1;
                    }
                    for (int cb = 0; cb < Tc; cb += 64) {
                        const int r = cb + l;
                        const int p = flat_parent<G>(M.map, excl, c, cb);
                        const int jj = r - __shfl(excl, p, 64);
                        const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
                        const int nsrc = __shfl(pm.nsrc, p, 64);
                        const int e0 = __shfl(pm.e0, p, 64);
                        const uint32_t pp = (uint32_t)__shfl((int)path, p, 64);
                        const uint32_t tag = (uint32_t)__shfl((int)one, p, 64);
                        const int sx = jj < nsrc ? select_bit_fast(src, jj) : e0;
                        // append the step in the first empty field (level)
                        const uint32_t child = (pp & ~(31u << (5 * level))) | ((uint32_t)sx << (5 * level));
                        if (r < Tc) st32<G>(fb + nn + r, child | tag | PATHF);
                    }
                    nn += Tc;
                    T += (uint32_t)Tc;
                    if ((int)T > heavy_t) return -2;
                }
                sync<G>();
                if (T == 0) break;
                uint32_t* t = fa; fa = fb; fb = t;
                n = nn;
                ++level;
                if (level <= 2) STAMP(6); else if (level == 3) STAMP(7); else STAMP(8);
            }
            fin = fa;
            if (level == 0) {
                nfin = 0;
            } else if (level == 4) {
                nfin = n;
            } else {
                for (int b = 0; b < n; b += 64) {   // parent had one move (order kept)
                    const int i = b + l;
                    const uint32_t e = i < n ? ld32<G>(fa + i) : 0u;
                    const bool rec = i < n && (e & FLAG1);
                    const uint64_t bm = ballot(rec);
                    sync<G>();
                    if (rec) st32<G>(fa + nfin + mask_prefix(bm), e);
                    nfin += __popcll(bm);
                    sync<G>();
                }
            }
            STAMP(9);
            fin_out = fin;
            return nfin;
        }
        if (l == 0) st32<G>(fa, KEY_EMPTY4);
        sync<G>();
        int n = 1, level = 0;
        while (level < 4) {
            clear_tab<G>(M);
            inserted = 0;
            int nn = 0;
            uint32_t T = 0;
            for (int b = 0; b < n; b += 64) {
                const int i = b + l;
                const bool live = i < n;
                const uint32_t pkey = live ? ld32<G>(fa + i) & KEYMASK : KEY_EMPTY4;
                const Moves pm = node_moves(R, rebuild(R, pkey, d), d, okd);
                const int cnt = live ? pm.n : 0;
                auto kfn = [&](int p, int s) -> uint32_t {
                    return key_insert((uint32_t)__shfl((int)pkey, p, 64), rel_of(s, R.player));
                };
                uint32_t tot;
                if (!expand_flat<G>(M, pm, cnt, pm.n == 1 ? FLAG1 : 0u, T, kfn, fb, nn, inserted, tot)) {
                    STAMP_COUNT(25);
                    return -1;
                }
                T += tot;
                if ((int)T > heavy_t) return -2;
            }
            if (T == 0) break;
            uint32_t* t = fa; fa = fb; fb = t;
            n = nn;
            ++level;
        }
        // records: the deepest level; below depth 4 only nodes whose parent had one move
        fin = fa;
        if (level == 0) {
            nfin = 0;
        } else if (level == 4) {
            nfin = n;
        } else {
            for (int b = 0; b < n; b += 64) {   // compact flagged nodes in place (order kept)
                const int i = b + l;
                const uint32_t e = i < n ? ld32<G>(fa + i) : 0u;
                const bool rec = i < n && (e & FLAG1);
                const uint64_t bm = ballot(rec);
                sync<G>();
                if (rec) st32<G>(fa + nfin + mask_prefix(bm), e);
                nfin += __popcll(bm);
                sync<G>();
            }
        }
    }
    fin_out = fin;
    return nfin;
}

// write the job's records (keys in `fin`) as boards at rows base..base+nfin-1
template <bool G>
BGX_DEV void emit_records(const MovegenArgs& a, int j, const JobIn& in, const uint32_t* fin, int nfin, int base,
                          int b0 = 0, int bstep = 64) {
    const bool dbl = in.d0 == in.d1;
    for (int b = b0; b < nfin; b += bstep) {
        const int i = b + lane_id();
        if (i < nfin) {
            const uint32_t e = ld32<G>(fin + i);
            const Node n = !dbl ? nd_board(in.R, e)
                                : ((e & PATHF) ? path_board(in.R, e & KEYMASK, in.d0) : rebuild(in.R, e & KEYMASK, in.d0));
            emit_one(a, j, in.R, n, i, base);
        }
    }
}

// A doubles job by path (doubles_by_path) as job_records + emit_records, except
// when the depth-4 list outgrows the slice: then the leaves are written
// straight to the output from the level-3 list -- the level-3 parents once to
// count the leaves (the output rows are reserved for them), once to expand and
// emit them in first-reach order, each leaf's board built from its path. So a
// job with hundreds of results (1-1 / 2-2 with many movable checkers: the 2-ply
// replies' usual tier-2 jobs) stays in tier 1. Same records. -1: a level-1..3
// list outgrew the slice (tier 2).
template <bool G>
BGX_DEV int path_doubles_emit(const MovegenArgs& a, int j, const JobIn& in, const Mem& M, FlatCursor& fc) {
    const Root& R = in.R;
    const int l = lane_id();
    const int d = in.d0;
    const uint32_t okd = ok_mask(R.block, d, R.player);
    uint32_t* fa = M.pa ? M.pa : M.fa;
    uint32_t* fb = M.pa ? M.pb : M.fb;
    const int PFc = M.pa ? M.PF : M.F;
    if (l == 0) st32<G>(fa, PATH_EMPTY);
    sync<G>();
    // a parent's filtered move list (lane-local): node, bar entry, first-reach filter
    auto parent = [&](uint32_t path, Moves& pm, uint32_t& one) {
        uint32_t bad, occ;
        const uint32_t nbar = path_state(R, path, d, okd, bad, occ);
        pm = path_moves(R, nbar, occ, d, okd);
        one = pm.n == 1 ? FLAG1 : 0u;
        pm.src &= ~bad;
        pm.nsrc = __popc(pm.src);
    };
    int n = 1, level = 0;
    bool stream4 = false;   // the depth-4 list would outgrow the slice: stream the leaves
    while (level < 4) {
        int nn = 0;
        for (int b = 0; b < n; b += 64) {
            const int i = b + l;
            const bool live = i < n;
            const uint32_t path = live ? ld32<G>(fa + i) & KEYMASK : PATH_EMPTY;
            Moves pm;
            uint32_t one;
            parent(path, pm, one);
            const int c = live ? pm.nsrc + (pm.e0 >= 0 ? 1 : 0) : 0;
            const int incl = wave_incl_scan(c);
            const int excl = incl - c;
            const int Tc = lane63(incl);
            if (n_out_check(nn, Tc, PFc)) {
                if (level < 3) return -1;
                stream4 = true;
                break;
            }
            for (int cb = 0; cb < Tc; cb += 64) {
                const int r = cb + l;
                const int p = flat_parent<G>(M.map, excl, c, cb);
                const int jj = r - __shfl(excl, p, 64);
                const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
                const int nsrc = __shfl(pm.nsrc, p, 64);
                const int e0 = __shfl(pm.e0, p, 64);
                const uint32_t pp = (uint32_t)__shfl((int)path, p, 64);
                const uint32_t tag = (uint32_t)__shfl((int)one, p, 64);
                const int sx = jj < nsrc ? select_bit_fast(src, jj) : e0;
                const uint32_t child = (pp & ~(31u << (5 * level))) | ((uint32_t)sx << (5 * level));
                if (r < Tc) st32<G>(fb + nn + r, child | tag | PATHF);
            }
            nn += Tc;
        }
        sync<G>();
        if (stream4 || nn == 0) break;
        uint32_t* t = fa; fa = fb; fb = t;
        n = nn;
        ++level;
    }
    if (!stream4) {
        // the deepest level; below depth 4 its nodes whose parent had one move
        // (none at level 0), as job_records
        int nfin = level == 4 ? n : 0;
        if (level > 0 && level < 4) {
            for (int b = 0; b < n; b += 64) {
                const int i = b + l;
                const uint32_t e = i < n ? ld32<G>(fa + i) : 0u;
                const bool rec = i < n && (e & FLAG1);
                const uint64_t bm = ballot(rec);
                sync<G>();
                if (rec) st32<G>(fa + nfin + mask_prefix(bm), e);
                nfin += __popcll(bm);
                sync<G>();
            }
        }
        const int base = begin_emit(a, j, nfin, fc);
        if (base >= 0) emit_records<G>(a, j, in, fa, nfin, base);
        return nfin;
    }
    // stream the leaves of the n level-3 parents in fa: count them
    int T4 = 0;
    {
        for (int b = 0; b < n; b += 64) {
            const int i = b + l;
            const uint32_t path = i < n ? ld32<G>(fa + i) & KEYMASK : PATH_EMPTY;
            Moves pm;
            uint32_t one;
            parent(path, pm, one);
            T4 += lane63(wave_incl_scan(i < n ? pm.nsrc + (pm.e0 >= 0 ? 1 : 0) : 0));
        }
    }
    const int base = begin_emit(a, j, T4, fc);
    if (base < 0) return T4;   // the flat buffer is full (flagged)
    int done = 0;
    for (int b = 0; b < n; b += 64) {
        const int i = b + l;
        const bool live = i < n;
        const uint32_t path = live ? ld32<G>(fa + i) & KEYMASK : PATH_EMPTY;
        Moves pm;
        uint32_t one;
        parent(path, pm, one);
        const int c = live ? pm.nsrc + (pm.e0 >= 0 ? 1 : 0) : 0;
        const int incl = wave_incl_scan(c);
        const int excl = incl - c;
        const int Tc = lane63(incl);
        for (int cb = 0; cb < Tc; cb += 64) {
            const int r = cb + l;
            const int p = flat_parent<G>(M.map, excl, c, cb);
            const int jj = r - __shfl(excl, p, 64);
            const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
            const int nsrc = __shfl(pm.nsrc, p, 64);
            const int e0 = __shfl(pm.e0, p, 64);
            const uint32_t pp = (uint32_t)__shfl((int)path, p, 64);
            const int sx = jj < nsrc ? select_bit_fast(src, jj) : e0;
            const uint32_t leaf = (pp & ~(31u << 15)) | ((uint32_t)sx << 15);
            if (r < Tc) emit_one(a, j, R, path_board(R, leaf, d), done + r, base);
        }
        done += Tc;
    }
    sync<G>();
    return T4;
}

// The six doubles rolls (d, d) of one root in one wave (two_ply.py:114-133),
// for a path-mode root (doubles_by_path: no node of any of its six trees can
// bear off). The trees expand level by level TOGETHER: a level's parents of
// all dice form one flat sequence (die-major; each list entry carries its die
// above the path), so the shallow levels -- one root and ~8 parents per die --
// fill the 64 lanes instead of running six nearly empty rounds, and the root
// is decoded once. A die whose next level is empty is finished from the
// current list (its nodes whose parent had one move, as job_records); the
// depth-4 leaves are counted per die, reserved and written straight to the
// output (as path_doubles_emit). Same records, offsets and counts per job as
// six per-roll jobs. cntd: 8 words of LDS. Returns the dice (bit d - 1) left to
// per-roll jobs: all six when the root is not in path mode, the unfinished
// ones when a level outgrows the slice's list.
constexpr uint32_t DIE_SHIFT = 20;   // list entry: path | die << 20 | PATHF | FLAG1
// index in the 21 DICE_ROLLS of the q-th non-doubles roll (the doubles sit at 0, 6, 11, 15, 18, 20)
BGX_DEV int nd_roll_q21(int q) { return q + 1 + (q >= 5) + (q >= 9) + (q >= 12) + (q >= 14); }
BGX_DEV int dbl_q21(int d) { return (d - 1) * 7 - ((d - 1) * d) / 2; }   // (d, d), d = 1..6

template <bool G>
BGX_DEV uint32_t board_dbl_emit(const MovegenArgs& a, int j0, const JobIn& in, const Mem& M, FlatCursor& fc,
                                uint32_t* cntd) {
    const Root& R = in.R;
    const int l = lane_id();
    if (!doubles_by_path(R) || M.force_table) return 0x3Fu;
    uint32_t* fa = M.pa;
    uint32_t* fb = M.pb;
    const int PFc = M.PF;
    const uint32_t ENTRY = KEYMASK | (7u << DIE_SHIFT);
    if (l < 6) st32<G>(fa + l, PATH_EMPTY | ((uint32_t)(l + 1) << DIE_SHIFT));
    // lane d (1..6): die d's first entry and entry count in the current list
    int dfirst = l >= 1 && l <= 6 ? l - 1 : 0, dcount = l >= 1 && l <= 6 ? 1 : 0;
    uint32_t done = 0u;   // dice finished (bit d - 1)
    int n = 6;
    sync<G>();
    for (int level = 0;; ++level) {
        const bool leaves = level == 3;   // this level's children are the records
        if (l < 8) st32<G>(cntd + l, 0u);
        sync<G>();
        // one parent per lane: its die, filtered move list and child count
        auto parent = [&](int i, uint32_t& e, int& d, Moves& pm, uint32_t& one) -> int {
            const bool live = i < n;
            e = live ? ld32<G>(fa + i) & ENTRY : (PATH_EMPTY | (1u << DIE_SHIFT));
            d = (int)((e >> DIE_SHIFT) & 7u);
            const uint32_t okd = ok_mask(R.block, d, R.player);
            uint32_t bad, occ;
            const uint32_t nbar = path_state(R, e & KEYMASK, d, okd, bad, occ);
            pm = path_moves(R, nbar, occ, d, okd);
            one = pm.n == 1 ? FLAG1 : 0u;
            pm.src &= ~bad;
            pm.nsrc = __popc(pm.src);
            return live ? pm.nsrc + (pm.e0 >= 0 ? 1 : 0) : 0;
        };
        int nn = 0;
        bool ovf = false;
        for (int b = 0; b < n; b += 64) {
            uint32_t e, one;
            int d;
            Moves pm;
            const int c = parent(b + l, e, d, pm, one);
            if (c > 0) atomicAdd(cntd + d, (uint32_t)c);
            const int incl = wave_incl_scan(c);
            const int excl = incl - c;
            const int Tc = lane63(incl);
            if (!leaves) {
                if (n_out_check(nn, Tc, PFc)) {
                    ovf = true;
                    break;
                }
                for (int cb = 0; cb < Tc; cb += 64) {
                    const int r = cb + l;
                    const int p = flat_parent<G>(M.map, excl, c, cb);
                    const int jj = r - __shfl(excl, p, 64);
                    const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
                    const int nsrc = __shfl(pm.nsrc, p, 64);
                    const int e0 = __shfl(pm.e0, p, 64);
                    const uint32_t pp = (uint32_t)__shfl((int)e, p, 64);
                    const uint32_t tag = (uint32_t)__shfl((int)one, p, 64);
                    const int sx = jj < nsrc ? select_bit_fast(src, jj) : e0;
                    const uint32_t child = (pp & ~(31u << (5 * level))) | ((uint32_t)sx << (5 * level));
                    if (r < Tc) st32<G>(fb + nn + r, child | tag | PATHF);
                }
            }
            nn += Tc;
        }
        sync<G>();
        if (ovf) return ~done & 0x3Fu;
        const int cd = l >= 1 && l <= 6 ? (int)ld32<G>(cntd + l) : 0;   // lane d: die d's children
        // dice whose tree ends here: their records are this level's nodes whose
        // parent had one move (none at level 0)
        uint32_t fin = (uint32_t)(ballot(l >= 1 && l <= 6 && cd == 0) >> 1) & ~done & 0x3Fu;
        while (fin) {
            const int d = __ffs(fin);
            fin &= fin - 1u;
            int f0 = __builtin_amdgcn_readlane(dfirst, d), fcnt = __builtin_amdgcn_readlane(dcount, d);
            if (BGX_DBL_GUARD && (f0 < 0 || fcnt < 0 || f0 + fcnt > n)) {
                if (l == 0) atomicOr(a.err_flags, 0x100u);
                f0 = fcnt = 0;
            }
            const int j = j0 + dbl_q21(d);
            int nrec = 0;
            if (level > 0)
                for (int b = 0; b < fcnt; b += 64) {
                    const bool rec = b + l < fcnt && (ld32<G>(fa + f0 + b + l) & FLAG1);
                    nrec += __popcll(ballot(rec));
                }
            const int base = begin_emit(a, j, nrec, fc);
            if (base >= 0 && nrec > 0) {
                int k0 = 0;
                for (int b = 0; b < fcnt; b += 64) {
                    const uint32_t e = b + l < fcnt ? ld32<G>(fa + f0 + b + l) : 0u;
                    const bool rec = b + l < fcnt && (e & FLAG1);
                    const uint64_t bm = ballot(rec);
                    const int kk = k0 + mask_prefix(bm);
                    bool okw = true;
                    if (BGX_DBL_GUARD && rec && (kk >= nrec || base + kk >= a.flat_cap)) {
                        atomicOr(a.err_flags, 0x200u);
                        okw = false;
                    }
                    if (rec && okw) emit_one(a, j, R, path_board(R, e & KEYMASK, d), kk, base);
                    k0 += __popcll(bm);
                }
            }
            done |= 1u << (d - 1);
        }
        if (done == 0x3Fu) return 0u;
        // lane d: die d's first child in the next level (children are die-major)
        const int cincl = wave_incl_scan(cd);
        if (!leaves) {
            uint32_t* t = fa; fa = fb; fb = t;
            n = nn;
            dfirst = cincl - cd;
            dcount = cd;
            continue;
        }
        // the leaves: every remaining die's rows, then the level-3 parents again,
        // each leaf written at its die's base + its index within the die
        int dbase = 0;
        for (uint32_t rem = ~done & 0x3Fu; rem; rem &= rem - 1u) {
            const int d = __ffs(rem);
            const int base = begin_emit(a, j0 + dbl_q21(d), __builtin_amdgcn_readlane(cd, d), fc);
            dbase = l == d ? base : dbase;
        }
        const int cfirst = cincl - cd;   // lane d: die d's first leaf in the flat order
        int done_r = 0;
        for (int b = 0; b < n; b += 64) {
            uint32_t e, one;
            int d;
            Moves pm;
            const int c = parent(b + l, e, d, pm, one);
            const int incl = wave_incl_scan(c);
            const int excl = incl - c;
            const int Tc = lane63(incl);
            for (int cb = 0; cb < Tc; cb += 64) {
                const int r = cb + l;
                const int p = flat_parent<G>(M.map, excl, c, cb);
                const int jj = r - __shfl(excl, p, 64);
                const uint32_t src = (uint32_t)__shfl((int)pm.src, p, 64);
                const int nsrc = __shfl(pm.nsrc, p, 64);
                const int e0 = __shfl(pm.e0, p, 64);
                const uint32_t pp = (uint32_t)__shfl((int)e, p, 64);
                const int pd = (int)((pp >> DIE_SHIFT) & 7u);
                const int base = __shfl(dbase, pd, 64), first = __shfl(cfirst, pd, 64);
                bool okw = true;
                if (BGX_DBL_GUARD) {
                    const int cnt = __shfl(cd, pd, 64), idx = done_r + r - first;
                    const bool badd = pd < 1 || pd > 6 || ((done >> (pd - 1)) & 1u);
                    if (r < Tc && (badd || idx < 0 || idx >= cnt || (base >= 0 && base + idx >= a.flat_cap))) {
                        atomicOr(a.err_flags, badd ? 0x400u : 0x800u);
                        okw = false;
                    }
                }
                const int sx = jj < nsrc ? select_bit_fast(src, jj) : e0;
                const uint32_t leaf = (pp & KEYMASK & ~(31u << 15)) | ((uint32_t)sx << 15);
                if (r < Tc && base >= 0 && okw)
                    emit_one(a, j0 + dbl_q21(pd), R, path_board(R, leaf, pd), done_r + r - first, base);
            }
            done_r += Tc;
        }
        sync<G>();
        return 0u;
    }
}

// LEAF: path doubles stream their leaves when the depth-4 list would outgrow
// the slice (path_doubles_emit); the large launches (pool / reply kernels) use
// it, the fused 1-ply kernel keeps job_records (its registers are at the cap)
template <bool G, bool LEAF = false>
BGX_DEV int run_job(const MovegenArgs& a, int j, const JobIn& in, const Mem& M, FlatCursor& fc,
                    int heavy_t = 0x7FFFFFFF) {
    if constexpr (LEAF) {
        if (in.d0 == in.d1 && doubles_by_path(in.R) && !M.force_table) return path_doubles_emit<G>(a, j, in, M, fc);
    }
    uint32_t* fin = nullptr;
    const int nfin = job_records<G>(in, M, fin, heavy_t);
    if (nfin < 0) return nfin;
    const int base = begin_emit(a, j, nfin, fc);
    if (base >= 0) emit_records<G>(a, j, in, fin, nfin, base);
    return nfin;
}

// ------------------------------------------------------------------ board-major replies (2-ply)
// two_ply.py:114-133 expands every roll of every candidate. The per-(root,
// roll) job above redoes the root analysis, its first-move lists and a
// mostly idle 64-lane emission for each of the 21 rolls; here one wave runs
// the 15 NON-DOUBLES rolls of a root together:
//  * each lane holds one FIRST move (die d, source s1), dice descending in
//    lane order; roll (H, L) takes its pass-0 parents (high die first) from
//    the die-H lanes and its pass-1 parents from the die-L lanes, so in lane
//    order a roll's pass-0 parents precede its pass-1 parents -- the
//    reference's (pass, i, j) enumeration (handle_non_doubles,
//    generate_all_moves.py:23-68);
//  * a roll's children are expanded flat over its parent lanes (64 per
//    round, flat_parent) and its records appended to one list for the root;
//  * the root's records are written in one pass (all 64 lanes busy), and the
//    15 jobs get their offsets inside that block.
// Roots it applies to (the others return -1 and run as per-roll jobs):
//  - rule mode (nd_by_rule: nothing on the bar, >= 3 mover checkers outside
//    home): no node of the two-step tree is on the bar or bearing off; records
//    are filtered by nd_first exactly as job_records' rule branch;
//  - the mover on the bar: the only first move of a die is the bar entry; a
//    child's moves are the normal moves of the entered board (bar 1: the
//    entered checker is outside home, so no bear-off) or the second entry
//    (bar >= 2). The two passes' plays are distinct except one board: with
//    bar 1 the two chains (enter and move on with the other die) end on the
//    same point and are the same board iff neither entry point held a blot;
//    with bar >= 2 the two double entries are the same board. Every other
//    pair differs in the mover's checkers (an addition at e_H = x + H would
//    need a source x off the board). So a pass-1 play is dropped iff its key
//    equals that pass-0 play's key; nothing else needs a table.
// Keys (nd_key, the non-doubles record format) go to `list` roll-major, the
// rolls in DICE_ROLLS order (two_ply.py:10-32) without the doubles; lane q of
// `rcnt` = the record count of the q-th non-doubles roll. Returns the record
// count, or -1 (not applicable, more than 64 first moves, or the list is full).
constexpr int ND_ROLLS = 15;

template <int LISTCAP>
BGX_DEV int board_nd_records(const Root& R, uint32_t* map, uint32_t* list, int& rcnt) {
    const int l = lane_id();
    const bool p0 = R.player == 0;
    const bool onbar = R.bar > 0u;
    const bool rule = !onbar && nd_by_rule(R);
    rcnt = 0;
    if (!onbar && !rule) return -1;
    const uint32_t occ = occ24(R.m0, R.m1, R.m2);
    auto entry = [&](int d) -> int { return p0 ? d - 1 : 24 - d; };
    auto open = [&](int d) -> bool { return !((R.block >> entry(d)) & 1u); };
    // first moves per die (wave-uniform): die d owns lanes [st(d), st(d) + n(d)),
    // dice descending; the lane's die is the lowest d with st(d) <= lane
    int st = 0, dl = 6, kst = 0;
    uint32_t srcl = 0u;
#pragma unroll
    for (int d = 6; d >= 1; --d) {
        const uint32_t sd = rule ? occ & ok_mask(R.block, d, R.player) : (open(d) ? 1u : 0u);
        if (l >= st) {
            dl = d;
            srcl = sd;
            kst = st;
        }
        st += __popc(sd);
    }
    const int nf = st;
    if (nf > 64) return -1;
    const bool valid = l < nf;
    // the lane's first move: source s1 (24 = the bar), destination t1, hit h1,
    // and the occupancy of the board after it (the child's normal-move sources)
    int s1 = 24, t1 = 0;
    uint32_t base2 = 0u;
    if (valid) {
        if (rule) {
            s1 = select_bit_fast(srcl, l - kst);
            t1 = p0 ? s1 + dl : s1 - dl;
            const uint32_t last1 = nib(R.m0, R.m1, R.m2, s1) == 1u ? 1u << s1 : 0u;
            base2 = (occ & ~last1) | (1u << t1);
        } else {
            t1 = entry(dl);
            base2 = occ | (1u << t1);
        }
    }
    const bool h1 = valid && ((R.blot >> t1) & 1u);
    const uint32_t pinfo = (uint32_t)s1 | ((uint32_t)t1 << 5) | (h1 ? 1u << 10 : 0u);
    const bool child_bar = R.bar >= 2u;   // after one entry the mover is still on the bar
    int total = 0, q = 0;
    for (int Ld = 1; Ld <= 5; ++Ld) {
        for (int Hd = Ld + 1; Hd <= 6; ++Hd, ++q) {
            const bool isH = valid && dl == Hd, isL = valid && dl == Ld;
            const uint32_t okH = ok_mask(R.block, Hd, R.player), okL = ok_mask(R.block, Ld, R.player);
            uint32_t m2 = 0u;
            if (isH || isL) {
                if (child_bar) m2 = open(isH ? Ld : Hd) ? 1u << 24 : 0u;   // bit 24: the bar entry
                else m2 = base2 & (isH ? okL : okH);
            }
            const bool two1 = ballot(isH && m2 != 0u) != 0ull;
            const bool two2 = ballot(isL && m2 != 0u) != 0ull;
            const int nH = rule ? __popc(occ & okH) : (open(Hd) ? 1 : 0);
            int cq = 0;
            if (two1 || (nH != 1 && two2)) {
                // 2-move records
                if (rule && isL) {   // a pass-1 parent adds only its chain or reverse-chain child
                    const int rv = p0 ? s1 - Hd : s1 + Hd;
                    m2 &= (1u << t1) | ((rv >= 0 && rv < 24) ? 1u << rv : 0u);
                }
                // bar mode: the pass-0 play that a pass-1 play can repeat (see above)
                uint32_t K0 = ND_DROP;
                if (!rule) {
                    const int eH = entry(Hd), eL = entry(Ld);
                    const bool hH = (R.blot >> eH) & 1u;
                    if (child_bar) {
                        if (open(Hd) && open(Ld))
                            K0 = nd_key(24u, (uint32_t)eH, hH, 24u, (uint32_t)eL, ((R.blot >> eL) & 1u) != 0u);
                    } else if (open(Hd) && ((okL >> eH) & 1u)) {
                        const int t2 = p0 ? eH + Ld : eH - Ld;
                        const uint32_t b2 = R.blot & ~(hH ? 1u << eH : 0u);
                        K0 = nd_key(24u, (uint32_t)eH, hH, (uint32_t)eH, (uint32_t)t2, ((b2 >> t2) & 1u) != 0u);
                    }
                }
                const int c = __popc(m2);
                const int incl = wave_incl_scan(c);
                const int excl = incl - c;
                const int T = lane63(incl);
                const uint32_t pi = pinfo | (isL ? 1u << 11 : 0u);
                for (int b = 0; b < T; b += 64) {
                    const int r = b + l;
                    const int p = flat_parent<false>(map, excl, c, b);
                    const int j = r - __shfl(excl, p, 64);
                    const uint32_t src2 = (uint32_t)__shfl((int)m2, p, 64);
                    const uint32_t ppi = (uint32_t)__shfl((int)pi, p, 64);
                    const uint32_t ps1 = ppi & 31u, pt1 = (ppi >> 5) & 31u;
                    const bool ph1 = (ppi >> 10) & 1u;
                    const int pp = (int)((ppi >> 11) & 1u);
                    const int s2 = (src2 >> 24) ? 24 : select_bit_fast(src2, j);
                    const int t2 = dest_of(R, s2, pp ? Hd : Ld);
                    const uint32_t blot2 = R.blot & ~(ph1 ? 1u << pt1 : 0u);
                    const bool h2 = t2 < 24 && ((blot2 >> t2) & 1u);
                    const uint32_t key = nd_key(ps1, pt1, ph1, (uint32_t)s2, (uint32_t)t2, h2);
                    const bool keep = rule ? nd_first(R, occ, pp, (int)ps1, (int)pt1, s2, t2, Hd, Ld)
                                           : !(pp == 1 && key == K0);
                    const bool sv = r < T && keep;
                    const uint64_t bm = ballot(sv);
                    const int ns = __popcll(bm);
                    if (total + cq + ns > LISTCAP) return -1;
                    if (sv) list[total + cq + mask_prefix(bm)] = key;
                    cq += ns;
                }
            } else {
                // singles: high-die singles, then low-die singles unless the high
                // die has exactly one move (handle_non_doubles 70-81; the pass-2 skip)
                const bool sv = isH || (isL && nH != 1);
                const uint64_t bm = ballot(sv);
                cq = __popcll(bm);
                if (total + cq > LISTCAP) return -1;
                if (sv) list[total + mask_prefix(bm)] = nd_key((uint32_t)s1, (uint32_t)t1, h1, 31u, 31u, false);
            }
            rcnt = l == q ? cq : rcnt;
            total += cq;
        }
    }
    wave_sync();
    return total;
}

// The same records, all 15 rolls' children as ONE flat sequence (roll-major,
// then parent lane, then move) cut into 64-child rounds, instead of one round
// trip per roll: a roll has ~40 children, so per-roll rounds ran half empty
// and the 15 dependent scan / parent-map / shuffle chains of a root were its
// latency. Each lane is a parent in the 5 rolls that pair its die with
// another; its children lists (m2, after the rule-mode pass-1 restriction) go
// to an LDS table [lane][partner die] and its first move to pinfo[lane]; a
// child finds its parent through the 64-word map (marks = start << 10 |
// roll << 6 | lane, + 1; a max-scan carries the latest start) and reads the
// two LDS words, so no shuffle is needed. Singles rolls (no 2-move play) give
// each eligible parent one child: the single itself. aux: >= 64 * 7 + 16
// words of LDS (the slice's second list).
template <int LISTCAP>
BGX_DEV int board_nd_records2(const Root& R, uint32_t* map, uint32_t* list, uint32_t* aux, int& rcnt) {
    const int l = lane_id();
    const bool p0 = R.player == 0;
    const bool onbar = R.bar > 0u;
    const bool rule = !onbar && nd_by_rule(R);
    rcnt = 0;
    if (!onbar && !rule) return -1;
    const uint32_t occ = occ24(R.m0, R.m1, R.m2);
    auto entry = [&](int d) -> int { return p0 ? d - 1 : 24 - d; };
    auto open = [&](int d) -> bool { return !((R.block >> entry(d)) & 1u); };
    uint32_t* m2tab = aux;              // [64][6]: lane's children sources with partner die dB (bit 24: bar entry)
    uint32_t* pinfo = aux + 64 * 6;     // [64]: s1 | t1 << 5 | h1 << 10 | die << 12
    uint32_t* rcl = aux + 64 * 7;       // [16]: records per roll
    uint32_t* k0tab = aux + 64 * 7 + 16;   // [16]: bar mode, the pass-0 play a pass-1 play of roll q repeats
    // first moves per die (wave-uniform): die d owns lanes [st(d), st(d) + n(d)), dice descending
    int st = 0, dl = 6, kst = 0;
    uint32_t srcl = 0u, nmask = 0u;     // nmask: bits 5(d-1): n(d)
#pragma unroll
    for (int d = 6; d >= 1; --d) {
        const uint32_t sd = rule ? occ & ok_mask(R.block, d, R.player) : (open(d) ? 1u : 0u);
        if (l >= st) {
            dl = d;
            srcl = sd;
            kst = st;
        }
        const int nd = __popc(sd);
        nmask |= (uint32_t)nd << (5 * (d - 1));
        st += nd;
    }
    const int nf = st;
    if (nf > 64) return -1;
    const bool valid = l < nf;
    int s1 = 24, t1 = 0;
    uint32_t base2 = 0u;
    if (valid) {
        if (rule) {
            s1 = select_bit_fast(srcl, l - kst);
            t1 = p0 ? s1 + dl : s1 - dl;
            const uint32_t last1 = nib(R.m0, R.m1, R.m2, s1) == 1u ? 1u << s1 : 0u;
            base2 = (occ & ~last1) | (1u << t1);
        } else {
            t1 = entry(dl);
            base2 = occ | (1u << t1);
        }
    }
    const bool h1 = valid && ((R.blot >> t1) & 1u);
    const bool child_bar = R.bar >= 2u;
    if (l < 16) rcl[l] = 0u;
    // children lists per partner die: counts before (cu) and after (cr) the
    // rule-mode pass-1 restriction, 5 bits each, packed by partner die
    uint32_t cu_pack = 0u, cr_pack = 0u;
    for (int dB = 1; dB <= 6; ++dB) {
        uint32_t m2 = 0u;
        if (valid && dB != dl) {
            if (child_bar) m2 = open(dB) ? 1u << 24 : 0u;
            else m2 = base2 & ok_mask(R.block, dB, R.player);
        }
        cu_pack |= (uint32_t)(__popc(m2 & 0xFFFFFFu) + (m2 >> 24)) << (5 * (dB - 1));
        if (rule && dB > dl) {   // this lane is a pass-1 parent of (dB, dl): chain / reverse chain only
            const int rv = p0 ? s1 - dB : s1 + dB;
            m2 &= (1u << t1) | ((rv >= 0 && rv < 24) ? 1u << rv : 0u);
        }
        cr_pack |= (uint32_t)(__popc(m2 & 0xFFFFFFu) + (m2 >> 24)) << (5 * (dB - 1));
        m2tab[l * 6 + dB - 1] = m2;
    }
    pinfo[l] = (uint32_t)s1 | ((uint32_t)t1 << 5) | (h1 ? 1u << 10 : 0u) | ((uint32_t)dl << 12);
    // per roll: the mode (2-move records or singles) and the children counts;
    // each lane keeps, per partner die pd, its children's flat start in roll
    // (pd, its die) as 1 << 14 | roll << 10 | start (16 bits; two partners per word)
    uint32_t single_mask = 0u, mk01 = 0u, mk23 = 0u, mk45 = 0u;
    int total = 0, q = 0;
    for (int Ld = 1; Ld <= 5; ++Ld) {
        for (int Hd = Ld + 1; Hd <= 6; ++Hd, ++q) {
            const bool isH = valid && dl == Hd, isL = valid && dl == Ld;
            const int cuH = (int)((cu_pack >> (5 * (Ld - 1))) & 31u);   // a die-H lane's children with L
            const int cuL = (int)((cu_pack >> (5 * (Hd - 1))) & 31u);   // a die-L lane's children with H
            const bool two1 = ballot(isH && cuH > 0) != 0ull;
            const bool two2 = ballot(isL && cuL > 0) != 0ull;
            const int nH = (int)((nmask >> (5 * (Hd - 1))) & 31u);
            const bool two = two1 || (nH != 1 && two2);
            int c = 0;
            if (two) {
                c = isH ? (int)((cr_pack >> (5 * (Ld - 1))) & 31u) : (isL ? (int)((cr_pack >> (5 * (Hd - 1))) & 31u) : 0);
            } else {
                single_mask |= 1u << q;
                c = (isH || (isL && nH != 1)) ? 1 : 0;
            }
            const int incl = wave_incl_scan(c);
            const int start = total + incl - c;
            if (c > 0) {   // this lane's start in roll q (partner die = the roll's other die)
                const int pd = isH ? Ld : Hd;
                const uint32_t v = (1u << 14 | (uint32_t)q << 10 | ((uint32_t)start & 1023u)) << (16 * ((pd - 1) & 1));
                mk01 |= pd <= 2 ? v : 0u;
                mk23 |= pd == 3 || pd == 4 ? v : 0u;
                mk45 |= pd >= 5 ? v : 0u;
            }
            total += lane63(incl);
            if (!rule && two && l == 0) {
                // bar mode: the pass-0 play that a pass-1 play of this roll can repeat
                uint32_t K0 = ND_DROP;
                const int eH = entry(Hd), eL = entry(Ld);
                const bool hH = (R.blot >> eH) & 1u;
                if (child_bar) {
                    if (open(Hd) && open(Ld))
                        K0 = nd_key(24u, (uint32_t)eH, hH, 24u, (uint32_t)eL, ((R.blot >> eL) & 1u) != 0u);
                } else if (open(Hd) && ((ok_mask(R.block, Ld, R.player) >> eH) & 1u)) {
                    const int t2c = p0 ? eH + Ld : eH - Ld;
                    const uint32_t b2 = R.blot & ~(hH ? 1u << eH : 0u);
                    K0 = nd_key(24u, (uint32_t)eH, hH, (uint32_t)eH, (uint32_t)t2c, ((b2 >> t2c) & 1u) != 0u);
                }
                k0tab[q] = K0;
            }
        }
    }
    if (total > 1023) return -1;   // (10-bit starts; far above any root's children)
    // the flat rounds
    int n_out = 0;
    uint32_t carry = 0u;
    for (int b = 0; b < total; b += 64) {
        // marks of the parents whose children start in this round
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t w = k < 2 ? mk01 : (k < 4 ? mk23 : mk45);
            const uint32_t e = (w >> (16 * (k & 1))) & 0xFFFFu;
            const uint32_t s = e & 1023u;
            if ((e >> 14) && (int)s >= b && (int)s < b + 64)
                map[s - b] = ((s << 10) | (((e >> 10) & 15u) << 6) | (uint32_t)l) + 1u;
        }
        wave_sync();
        uint32_t mk = map[l];
        map[l] = 0u;
        mk = (uint32_t)wave_incl_max((int)mk);
        mk = mk ? mk : carry;
        carry = (uint32_t)lane63((int)mk);
        const int r = b + l;
        const uint32_t code = (mk - 1u) & 1023u;
        const int qq = (int)(code >> 6), p = (int)(code & 63u);
        const int jj = r - (int)((mk - 1u) >> 10);
        // the roll's dice (DICE_ROLLS order of the non-doubles): L from the group starts 0, 5, 9, 12, 14
        const int L = 1 + (qq >= 5) + (qq >= 9) + (qq >= 12) + (qq >= 14);
        const int H = L + 1 + qq - ((L - 1) * (12 - L)) / 2;
        const uint32_t pi = pinfo[p];
        const uint32_t ps1 = pi & 31u, pt1 = (pi >> 5) & 31u;
        const bool ph1 = (pi >> 10) & 1u;
        const int pdl = (int)(pi >> 12);
        const int pp = pdl == L ? 1 : 0;   // pass 1: the parent moved the low die first
        uint32_t key;
        bool keep = true;
        if ((single_mask >> qq) & 1u) {
            key = nd_key(ps1, pt1, ph1, 31u, 31u, false);
        } else {
            const uint32_t src2 = m2tab[p * 6 + (pp ? H : L) - 1];
            const int s2 = (src2 >> 24) ? 24 : select_bit_fast(src2, jj);
            const int t2 = dest_of(R, s2, pp ? H : L);
            const uint32_t blot2 = R.blot & ~(ph1 ? 1u << pt1 : 0u);
            const bool h2 = t2 < 24 && ((blot2 >> t2) & 1u);
            key = nd_key(ps1, pt1, ph1, (uint32_t)s2, (uint32_t)t2, h2);
            if (rule) {
                keep = nd_first(R, occ, pp, (int)ps1, (int)pt1, s2, t2, H, L);
            } else if (pp == 1) {
                keep = key != k0tab[qq];   // bar mode (board_nd_records)
            }
        }
        const bool sv = r < total && keep;
        const uint64_t bm = ballot(sv);
        const int ns = __popcll(bm);
        if (n_out + ns > LISTCAP) return -1;
        if (sv) {
            list[n_out + mask_prefix(bm)] = key;
            atomicAdd(&rcl[qq], 1u);
        }
        n_out += ns;
    }
    wave_sync();
    rcnt = l < ND_ROLLS ? (int)rcl[l] : 0;
    return n_out;
}

// OUT_PACKED_FLAT rows for n records (one global atomic per chunk of rows, as
// begin_emit); -1 = the flat buffer is full (flagged)
BGX_DEV int reserve_flat(const MovegenArgs& a, int n, FlatCursor& fc, int want) {
    int base = 0;
    if (cursor_take(fc, n, base)) return base;
    if (fc.wg) return wg_take(a, n, fc);
    if (want > a.flat_chunk) want = a.flat_chunk;
    const int grab = n > want ? n : want;
    if (lane_id() == 0) base = (int)atomicAdd(a.flat_count, (unsigned)grab);
    base = uniform(base);
    if (base + grab > a.flat_cap) {
        if (lane_id() == 0) atomicOr(a.err_flags, BGX_ERRF_FLAT_OVERFLOW);
        fc.left = fc.left2 = 0;
        return -1;
    }
    cursor_new_chunk(fc, base, n, grab);
    return base;
}

// ------------------------------------------------------------------ block-cooperative doubles
// Small launches (no more jobs than resident waves, e.g. the 1-ply step) are
// bound by their slowest job: a doubles roll with hundreds of results. A
// doubles job whose level outgrows HEAVY_T children in its wave is expanded
// again by the whole 16-wave block, level by level:
//  1. parents (2 per thread): rebuild, move list -> LDS (src mask, packed
//     extras, exclusive child prefix from a block scan), and a child -> parent
//     map (u16 per child);
//  2. children (one per thread per round): insert key << 32 | (ordinal << 1 |
//     parent-had-one-move) into a table sized for the level (dedup_insert's
//     CAS / atomicMin leave each key with its first-reach ordinal);
//  3. survivors = the occupied slots: set bit[ordinal], prefix-popcount the
//     bitmap, and each slot writes its key to the next frontier at its rank,
//     i.e. in first-reach order.
constexpr int BW = 16;                // waves per block
constexpr int NTH = 64 * BW;          // threads per block
constexpr int K_S = 4096;             // max table slots
constexpr int K_F = 2 * NTH;          // frontier capacity (2 parents per thread)
constexpr int K_TMAX = 16384;         // children per level
constexpr int HEAVY_T = 128;             // measured: 256 / 128 / 64 -> 128 best (1-ply)
struct CoopLds {
    unsigned long long tab[K_S];
    uint32_t fa[K_F], fb[K_F];
    uint32_t psrc[K_F], ppack[K_F], pexcl[K_F];
    uint16_t map[K_TMAX];
    uint32_t bits[K_TMAX / 32];
    uint16_t pre[K_TMAX / 32];
    uint32_t wsum[BW];
    uint32_t misc[8];                 // [0] inserted [1] record count [2] emit base [3] heavy mask
};
// block-wide exclusive scan of one value per thread (NWv waves, wsum[NWv] in
// LDS); `total` = block sum
template <int NWv>
BGX_DEV int block_excl_scan_w(uint32_t* wsum, int v, int& total) {
    const int w = (int)threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane_id() == 63) wsum[w] = (uint32_t)incl;
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < NWv; ++k) {
        const int t = (int)wsum[k];
        before += k < w ? t : 0;
        total += t;
    }
    __syncthreads();
    return before + incl - v;
}
BGX_DEV int block_excl_scan(CoopLds& C, int v, int& total) { return block_excl_scan_w<BW>(C.wsum, v, total); }

// LDS of the path expansion alone (the fused kernel's tier 2 lays it over
// its scratch): KF parents / children per level, two parents per thread
template <int NWv, int KF> struct CoopPathLds {
    uint32_t fa[KF], fb[KF];
    uint32_t psrc[KF], ppack[KF], pexcl[KF];
    uint16_t map[KF];
    uint32_t wsum[NWv];
};

// The table-free path expansion (doubles_by_path) by a whole block: per level
// the parents' filtered move lists and child prefix, then one child per
// thread written straight to its first-reach slot (no dedup, no ranking).
// NWv waves, KF <= 2 * 64 * NWv parents / children per level (-1 beyond).
template <int NWv, int KF, typename L>
BGX_DEV int coop_doubles_path(const JobIn& in, L& C, uint32_t*& fin) {
    static_assert(KF <= 2 * 64 * NWv, "two parents per thread");
    constexpr int NTH = 64 * NWv;
    const Root& R = in.R;
    const int d = in.d0;
    const int t = (int)threadIdx.x, w = t >> 6;
    const uint32_t okd = ok_mask(R.block, d, R.player);
    uint32_t* fa = C.fa;
    uint32_t* fb = C.fb;
    if (t == 0) fa[0] = PATH_EMPTY;
    __syncthreads();
    int n = 1, level = 0;
    while (level < 4) {
        int c[2] = {0, 0};
        uint32_t src[2] = {0u, 0u}, pack[2] = {0u, 0u};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            if (hh * NTH + 64 * w < n) {        // wave-uniform
                const int i = hh * NTH + t;
                const uint32_t path = i < n ? fa[i] & KEYMASK : PATH_EMPTY;
                uint32_t bad, occ;
                const uint32_t nbar = path_state(R, path, d, okd, bad, occ);
                const Moves pm = path_moves(R, nbar, occ, d, okd);
                const uint32_t ok = pm.src & ~bad;
                const int ns = __popc(ok);
                c[hh] = i < n ? ns + (pm.e0 >= 0 ? 1 : 0) : 0;
                src[hh] = ok;
                pack[hh] = (uint32_t)ns | ((uint32_t)(pm.e0 + 1) << 5) | (pm.n == 1 ? 1u << 15 : 0u);
            }
        }
        int tot2;
        const int ex2 = block_excl_scan_w<NWv>(C.wsum, c[0] | (c[1] << 16), tot2);
        const int T0 = tot2 & 0xFFFF, T = T0 + (tot2 >> 16);
        if (T == 0) break;                      // uniform
        if (T > KF) return -1;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int i = hh * NTH + t;
            if (i < n) {
                const int ex = hh ? T0 + (ex2 >> 16) : (ex2 & 0xFFFF);
                C.psrc[i] = src[hh];
                C.ppack[i] = pack[hh];
                C.pexcl[i] = (uint32_t)ex;
                for (int k = 0; k < c[hh]; ++k) C.map[ex + k] = (uint16_t)i;
            }
        }
        __syncthreads();
        for (int r = t; r < T; r += NTH) {
            const int p = (int)C.map[r];
            const uint32_t pk = C.ppack[p];
            const int jj = r - (int)C.pexcl[p];
            const int nsrc = (int)(pk & 31u);
            const int sx = jj < nsrc ? select_bit_fast(C.psrc[p], jj) : (int)((pk >> 5) & 31u) - 1;
            const uint32_t pp = fa[p] & KEYMASK;
            const uint32_t child = (pp & ~(31u << (5 * level))) | ((uint32_t)sx << (5 * level));
            fb[r] = child | (((pk >> 15) & 1u) ? FLAG1 : 0u) | PATHF;
        }
        __syncthreads();
        uint32_t* tmp = fa; fa = fb; fb = tmp;
        n = T;
        ++level;
    }
    fin = fa;
    if (level == 4) return n;
    if (level == 0) return 0;
    const int i0 = 2 * t;
    const uint32_t e0 = i0 < n ? fa[i0] : 0u, e1 = i0 + 1 < n ? fa[i0 + 1] : 0u;
    const int f0 = (i0 < n && (e0 & FLAG1)) ? 1 : 0, f1 = (i0 + 1 < n && (e1 & FLAG1)) ? 1 : 0;
    int nf;
    const int pos = block_excl_scan_w<NWv>(C.wsum, f0 + f1, nf);
    if (f0) fb[pos] = e0;
    if (f1) fb[pos + f0] = e1;
    __syncthreads();
    fin = fb;
    return nf;
}

// returns the record count (records in `fin`), -1 = overflow (tier 3)
BGX_DEV int coop_doubles(const JobIn& in, CoopLds& C, uint32_t*& fin, bool force_table = false) {
    if (doubles_by_path(in.R) && !force_table) return coop_doubles_path<BW, K_F>(in, C, fin);
    const Root& R = in.R;
    const int d = in.d0;
    const int t = (int)threadIdx.x, l = lane_id();
    const uint32_t okd = ok_mask(R.block, d, R.player);
    uint32_t* fa = C.fa;
    uint32_t* fb = C.fb;
    if (t == 0) fa[0] = KEY_EMPTY4;
    __syncthreads();
    int n = 1, level = 0;
    while (level < 4) {
        // 1. parents t and t + NTH (waves past the level skip the work)
        const int w = t >> 6;
        int c[2] = {0, 0};
        uint32_t src[2] = {0u, 0u}, pack[2] = {0u, 0u};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            if (hh * NTH + 64 * w < n) {        // wave-uniform
                const int i = hh * NTH + t;
                const uint32_t pkey = i < n ? fa[i] & KEYMASK : KEY_EMPTY4;
                const Moves pm = node_moves(R, rebuild(R, pkey, d), d, okd);
                c[hh] = i < n ? pm.n : 0;
                src[hh] = pm.src;
                pack[hh] = (uint32_t)pm.nsrc | ((uint32_t)(pm.e0 + 1) << 5) | ((uint32_t)(pm.e1 + 1) << 10) |
                           (pm.n == 1 ? 1u << 15 : 0u);
            }
        }
        // one block scan of both halves (16-bit fields: T <= K_TMAX < 2^15)
        int tot2;
        const int ex2 = block_excl_scan(C, c[0] | (c[1] << 16), tot2);
        const int T0 = tot2 & 0xFFFF, T = T0 + (tot2 >> 16);
        if (T == 0) break;                      // uniform
        if (T > K_TMAX) return -1;
        int S = 64;
        while (S < 2 * T && S < K_S) S <<= 1;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int i = hh * NTH + t;
            if (i < n) {
                const int ex = hh ? T0 + (ex2 >> 16) : (ex2 & 0xFFFF);
                C.psrc[i] = src[hh];
                C.ppack[i] = pack[hh];
                C.pexcl[i] = (uint32_t)ex;
                for (int k = 0; k < c[hh]; ++k) C.map[ex + k] = (uint16_t)i;
            }
        }
        for (int i = t; i < S; i += NTH) C.tab[i] = EMPTY64;
        const int nwd = (T + 31) >> 5;
        for (int i = t; i < nwd; i += NTH) C.bits[i] = 0u;
        if (t == 0) C.misc[0] = 0u;
        __syncthreads();
        // 2. children
        Mem M;
        M.tab = C.tab;
        M.S = S;
        int fresh_n = 0;
        for (int b = 0; b < T; b += NTH) {     // uniform trip count
            if (b + 64 * w >= T) break;        // wave-uniform: no children left for this wave
            const int r = b + t;
            const bool act = r < T;
            const int p = act ? (int)C.map[r] : 0;
            const uint32_t pk = C.ppack[p];
            const int jj = r - (int)C.pexcl[p];
            const int nsrc = (int)(pk & 31u);
            const int sx = jj < nsrc ? select_bit_fast(C.psrc[p], jj)
                                     : (jj == nsrc ? (int)((pk >> 5) & 31u) - 1 : (int)((pk >> 10) & 31u) - 1);
            const uint32_t key = key_insert(fa[p] & KEYMASK, rel_of(sx, R.player));
            const uint32_t ordw = ((uint32_t)r << 1) | ((pk >> 15) & 1u);
            bool fresh;
            dedup_insert<false>(M, act, key, ordw, fresh);
            fresh_n += __popcll(ballot(fresh));
        }
        if (l == 0 && fresh_n) atomicAdd(&C.misc[0], (uint32_t)fresh_n);
        __syncthreads();
        if ((int)C.misc[0] > K_F) return -1;   // uniform
        // 3. survivors in ordinal order
        for (int i = t; i < S; i += NTH) {
            const unsigned long long v = C.tab[i];
            if (v != EMPTY64) {
                const uint32_t o = (uint32_t)v >> 1;
                atomicOr(&C.bits[o >> 5], 1u << (o & 31));
            }
        }
        __syncthreads();
        int nn;
        const int cw = t < nwd ? __popc(C.bits[t]) : 0;   // nwd <= K_TMAX / 32 = NTH / 2
        const int pw = block_excl_scan(C, cw, nn);
        if (t < nwd) C.pre[t] = (uint16_t)pw;
        __syncthreads();
        for (int i = t; i < S; i += NTH) {
            const unsigned long long v = C.tab[i];
            if (v != EMPTY64) {
                const uint32_t ow = (uint32_t)v, o = ow >> 1;
                const int rank = (int)C.pre[o >> 5] + __popc(C.bits[o >> 5] & ((1u << (o & 31)) - 1u));
                fb[rank] = (uint32_t)(v >> 32) | ((ow & 1u) ? FLAG1 : 0u);
            }
        }
        __syncthreads();
        uint32_t* tmp = fa; fa = fb; fb = tmp;
        n = nn;
        ++level;
    }
    fin = fa;
    if (level == 4) return n;
    if (level == 0) return 0;
    // below depth 4: only nodes whose parent had one move (order kept)
    const int i0 = 2 * t;
    const uint32_t e0 = i0 < n ? fa[i0] : 0u, e1 = i0 + 1 < n ? fa[i0 + 1] : 0u;
    const int f0 = (i0 < n && (e0 & FLAG1)) ? 1 : 0, f1 = (i0 + 1 < n && (e1 & FLAG1)) ? 1 : 0;
    int nf;
    const int pos = block_excl_scan(C, f0 + f1, nf);
    if (f0) fb[pos] = e0;
    if (f1) fb[pos + f0] = e1;
    __syncthreads();
    fin = fb;
    return nf;
}

// ------------------------------------------------------------------ kernels
template <int S>
BGX_DEV Mem lds_mem(unsigned long long* smem) {
    Mem M;
    M.tab = smem;
    M.F = Slice<S>::F;
    M.fa = (uint32_t*)(smem + S);
    M.fb = M.fa + M.F;
    M.map = M.fb + M.F;
    M.S = S;
    M.map[lane_id()] = 0u;
    wave_sync();
    return M;
}

BGX_DEV void push_ovf(const MovegenArgs& a, int j) {
    if (BGX_DBL_GUARD && (j < 0 || j >= job_count(a))) {
        atomicOr(a.err_flags, 0x4000u);
        return;
    }
    const unsigned slot = atomicAdd(a.ovf_count, 1u);
    if ((int)slot < a.ovf_cap) a.ovf_list[slot] = j;
    else atomicOr(a.err_flags, BGX_ERRF_OVF_LIST);
}

}  // namespace bgx
