// bgx_engine.h — K4 device code (lane RNG, reset, rewards, the lane env step), shared by
// the engine kernels (bgx_engine.hip) and the fused 1-ply lane kernel (bgx_fused.hip).
// Reference mapping: see the header comment of bgx_engine.hip.
#pragma once
#include "bgx_device.h"
#include "bgx_kernels.h"

namespace bgx {

static __constant__ float kRollProb[21] = {
    1.f / 36, 2.f / 36, 2.f / 36, 2.f / 36, 2.f / 36, 2.f / 36, 1.f / 36, 2.f / 36, 2.f / 36, 2.f / 36, 2.f / 36,
    1.f / 36, 2.f / 36, 2.f / 36, 2.f / 36, 1.f / 36, 2.f / 36, 2.f / 36, 1.f / 36, 2.f / 36, 1.f / 36};
static __constant__ double kRollProbD[21] = {
    1. / 36, 2. / 36, 2. / 36, 2. / 36, 2. / 36, 2. / 36, 1. / 36, 2. / 36, 2. / 36, 2. / 36, 2. / 36,
    1. / 36, 2. / 36, 2. / 36, 2. / 36, 1. / 36, 2. / 36, 2. / 36, 1. / 36, 2. / 36, 1. / 36};

BGX_DEV uint64_t lane_key(uint64_t seed, uint32_t gid) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(gid + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Dice streams. Normal mode: Philox4x32-10 keyed by (seed, global lane id),
// one counter per draw. Scripted mode (test hook, bgx_engine_set_dice): the
// lane's dice come from a table of single-die draws, consumed two per roll in
// order (np.random.randint(1, 7) twice, backgammon_env.py:310-311), and the
// counter is the table cursor; past the end a roll is (1, 2) and the engine
// raises BGX_ERRF_DICE_EXHAUSTED. Scripted lanes play greedy (no uniform).
struct DiceTab {
    const uint8_t* tab = nullptr;   // the lane's row, or null
    uint32_t len = 0;
    BGX_DEV bool roll(uint64_t& ctr, int& a, int& b) const {   // false: past the end
        const bool ok = ctr + 1 < (uint64_t)len;
        a = ok ? (int)tab[ctr] : 1;
        b = ok ? (int)tab[ctr + 1] : 2;
        ctr += 2;
        return ok;
    }
};

struct LaneRng {
    uint64_t key, ctr;
    DiceTab dt;
    bool exhausted = false;
    BGX_DEV u32x4 next() { return philox(key, 0x5EED0000ull, ctr++); }
    BGX_DEV void roll(int& a, int& b) {
        if (dt.tab) { exhausted |= !dt.roll(ctr, a, b); return; }
        u32x4 r = next();
        a = die_from(r.x);
        b = die_from(r.y);
    }
    BGX_DEV void skip_uniform() { if (!dt.tab) ++ctr; }
};

// The same stream drawn by a half-wave (two game lanes per wavefront, one
// per half): lane k of the half evaluates counter base + k, draws come over
// by shuffles within the half.
struct HalfRng {
    uint64_t key, ctr, base;
    u32x4 batch;
    DiceTab dt;
    bool exhausted = false;
    BGX_DEV void refill() {
        base = ctr;
        batch = philox(key, 0x5EED0000ull, base + (uint64_t)(lane_id() & 31));
    }
    BGX_DEV u32x4 at(int k) const {   // counter base + k, k < 32 (uniform within the half)
        const int src = (lane_id() & 32) + k;
        return {(uint32_t)__shfl((int)batch.x, src, 64), (uint32_t)__shfl((int)batch.y, src, 64),
                (uint32_t)__shfl((int)batch.z, src, 64), (uint32_t)__shfl((int)batch.w, src, 64)};
    }
    BGX_DEV u32x4 next() {
        if (ctr - base >= 32u) refill();
        const u32x4 r = at((int)(ctr - base));
        ++ctr;
        return r;
    }
    BGX_DEV void roll(int& a, int& b) {
        if (dt.tab) { exhausted |= !dt.roll(ctr, a, b); return; }
        u32x4 r = next();
        a = die_from(r.x);
        b = die_from(r.y);
    }
    BGX_DEV void skip_uniform() { if (!dt.tab) ++ctr; }
};

// packed initial board (immutable_board.py:27-70): P1 {0:2, 11:5, 16:3, 18:5}, P2 {23:2, 12:5, 7:3, 5:5}
BGX_DEV void initial_packed(uint32_t* w) {
    w[0] = 0x2u;                       // P1 point 0: 2
    w[1] = 0x5u << 12;                 // P1 point 11: 5
    w[2] = (0x3u << 0) | (0x5u << 8);  // P1 points 16: 3, 18: 5
    w[3] = (0x5u << 20) | (0x3u << 28);// P2 points 5: 5, 7: 3
    w[4] = 0x5u << 16;                 // P2 point 12: 5
    w[5] = 0x2u << 28;                 // P2 point 23: 2
    w[6] = 0;
    w[7] = 0;
}

BGX_DEV void load_packed(const uint32_t* p, uint32_t* w) {
    const uint4 x = ((const uint4*)p)[0], y = ((const uint4*)p)[1];
    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
}
BGX_DEV void store_packed(uint32_t* p, const uint32_t* w) {
    ((uint4*)p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
    ((uint4*)p)[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
BGX_DEV void set_flag(uint32_t* w, int p) { w[6] = (w[6] & 0xFFFFu) | ((uint32_t)p << 16); }

// reset (backgammon_env.py:92-128); returns starter, leaves first dice in d0/d1
template <typename Rng>
BGX_DEV int new_game(Rng& rng, uint32_t* w, int& d0, int& d1) {
    initial_packed(w);
    int a, b;
    do { rng.roll(a, b); } while (a == b);
    const int starter = a < b ? 1 : 0;
    do { rng.roll(a, b); } while (a == b);
    d0 = a;
    d1 = b;
    set_flag(w, starter);
    return starter;
}

BGX_DEV uint32_t pts_word(const uint32_t* w, int pl, int k) { return pl ? w[3 + k] : w[k]; }

struct Outcome { float reward; int done, win_type, close, prime; };

// env_helper.py:113-242 on a packed board after `pl` moved
BGX_DEV Outcome judge(const uint32_t* w, int pl, uint32_t& flags) {
    Outcome o = {0.0f, 0, 0, 0, 0};
    const uint32_t s6 = w[6];
    const int op = 1 - pl;
    const uint32_t off_m = (s6 >> (8 + 4 * pl)) & 15u, off_o = (s6 >> (8 + 4 * op)) & 15u;
    const uint32_t bar_o = (s6 >> (4 * op)) & 15u;
    const uint32_t m0 = pts_word(w, pl, 0), m1 = pts_word(w, pl, 1), m2 = pts_word(w, pl, 2);
    const uint32_t o0 = pts_word(w, op, 0), o1 = pts_word(w, op, 1), o2 = pts_word(w, op, 2);
    const uint32_t occ_o = occ24(o0, o1, o2);
    const uint32_t home = pl == 0 ? 0xFC0000u : 0x3Fu;
    if (off_m >= 15u) {                                            // check_game_over
        o.done = 1;
        if (off_o == 0u && ((occ_o & home) || bar_o > 0u)) { o.reward = 2.5f; o.win_type = 3; }
        else if (off_o == 0u) { o.reward = 2.0f; o.win_type = 2; }
        else { o.reward = 1.0f; o.win_type = 1; }
        return o;
    }
    const uint32_t g = ge2_24(m0, m1, m2);
    float r = 0.0f;
    const bool closed = bar_o > 0u && (g & home) == home;          // is_closed_out
    if (closed && !(flags & (1u << pl))) {
        r += 0.30f;
        flags |= 1u << pl;
        o.close = 1;
    }
    const uint32_t run5 = g & (g >> 1) & (g >> 2) & (g >> 3) & (g >> 4) & 0xFFFFFu;
    bool prime = false;                                            // made_at_least_five_prime
    if (run5) {
        if (pl == 0) {
            const int s = __ffs(run5) - 1;
            prime = (occ_o >> (s + 5)) != 0u;
        } else {
            const int s = 31 - __clz(run5);
            prime = (occ_o & ((1u << s) - 1u)) != 0u;
        }
    }
    if (prime && !(flags & (4u << pl))) {
        r += 0.20f;
        flags |= 4u << pl;
        o.prime = 1;
    }
    o.reward = r;
    return o;
}


// A lane's state between env steps (EngineDev SoA fields of lane i).
struct LaneState {
    uint32_t w[8];        // board, indicator flag = player to move
    int p, d0, d1, steps;
    uint32_t flags, epi, rec, ep_first, harv, hepi;
    uint64_t ctr;         // Philox counter
};
BGX_DEV void lane_load(const EngineDev& e, int i, LaneState& s) {
    load_packed(e.rows + (size_t)i * 8, s.w);
    s.p = e.player[i];
    s.d0 = e.dice[2 * i];
    s.d1 = e.dice[2 * i + 1];
    s.steps = e.step[i];
    s.flags = e.flags[i];
    s.epi = e.epi[i];
    s.rec = e.rec_count[i];
    s.ep_first = e.ep_first[i];
    s.harv = e.harv[i];
    s.hepi = e.hepi ? e.hepi[i] : 0u;
    s.ctr = e.rng[i];
}
// everything but the board row (lane_advance writes that every step)
BGX_DEV void lane_store(const EngineDev& e, int i, const LaneState& s) {
    e.player[i] = (uint8_t)s.p;
    e.dice[2 * i] = (uint8_t)s.d0;
    e.dice[2 * i + 1] = (uint8_t)s.d1;
    e.step[i] = s.steps;
    e.flags[i] = s.flags;
    e.epi[i] = s.epi;
    e.rec_count[i] = s.rec;
    e.ep_first[i] = s.ep_first;
    e.rng[i] = s.ctr;
}

// the lane's scripted dice (bgx_engine_set_dice), or none
BGX_DEV DiceTab lane_dice(const EngineDev& e, int i) {
    DiceTab d;
    if (e.dice_tab) {
        d.tab = e.dice_tab + (size_t)i * (size_t)e.dice_len;
        d.len = (uint32_t)e.dice_len;
    }
    return d;
}

// One game lane's env step after its action is chosen (BackgammonEnv.step,
// backgammon_env.py:130-221, + the worker's Experience, worker.py:101-162):
// apply, judge, record, and on game end append the episode header and reset.
// action < 0 (or no legal move): pass. `nb` = the packed board (8 words) of
// candidate `action`, vs / va = V(s) / V(a), n_full = the full candidate count. The
// state update runs on every calling thread (a wave keeps its lane's state
// uniform in registers); only `lead` writes memory (record, episode header,
// the lane's board row).
template <typename Rng>
BGX_DEV void lane_advance(const EngineDev& e, int i, LaneState& s, Rng& rng, int action, const uint32_t* nb, float vs,
                          float va, int n_full, bool lead) {
    rng.ctr = s.ctr;
    const int n = n_full < e.max_legal ? n_full : e.max_legal;
    bool done = false;
    int win_type = 0, winner = -1;
    if (n == 0 || action < 0) {
        // pass (backgammon_env.py:139-151): no experience is recorded (worker.py:106-113)
        s.p ^= 1;
        rng.roll(s.d0, s.d1);
    } else {
        s.flags |= 16u << s.p;
        rng.skip_uniform();   // the sampling uniform (lane_uniform)
        const int a = action;
        const int mover = s.p;
        const int dd0 = s.d0, dd1 = s.d1;
        const Outcome o = judge(nb, mover, s.flags);
        done = o.done;
        if (done) { win_type = o.win_type; winner = mover; }
        else { s.p ^= 1; rng.roll(s.d0, s.d1); }
        // experience record (worker.py:149-156; Experience, episode.py:5-46): the
        // board before the move with the mover's indicator; the board after is
        // the next record's before-board or the header's final board
        const uint32_t rec = s.rec;
        if (lead) {
            if (rec - s.harv >= (uint32_t)e.R) atomicOr(e.err_flags, BGX_ERRF_RING_OVERFLOW);
            uint32_t* R = e.ring + ((size_t)i * e.R + (rec & (uint32_t)(e.R - 1))) * REC_WORDS;
            const uint32_t w6 = (s.w[6] & 0xFFFFu) | ((uint32_t)mover << 16);
            const uint32_t nm = (uint32_t)(n_full > 4095 ? 4095 : n_full);
            const uint32_t st = (uint32_t)(s.steps > 511 ? 511 : s.steps);
            ((uint4*)R)[0] = make_uint4(s.w[0], s.w[1], s.w[2], s.w[3]);
            ((uint4*)R)[1] = make_uint4(s.w[4], s.w[5], w6, __float_as_uint(vs));
            ((uint4*)R)[2] = make_uint4(__float_as_uint(va), __float_as_uint(o.reward),
                                        (uint32_t)a | (nm << 11) | (st << 23),
                                        (uint32_t)dd0 | ((uint32_t)dd1 << 3) | ((uint32_t)o.done << 6) |
                                            ((uint32_t)o.close << 7) | ((uint32_t)o.prime << 8) |
                                            ((uint32_t)mover << 9) | ((uint32_t)o.win_type << 10));
        }
        s.rec = rec + 1;
        for (int k = 0; k < 8; ++k) s.w[k] = nb[k];
    }
    ++s.steps;
    set_flag(s.w, s.p);
    if (done || s.steps >= e.max_steps) {
        if (lead) {
            // the header: the lane's own ring (fused engine: its workgroup
            // harvests it) or the engine's episode list
            uint32_t* h = nullptr;
            if (e.hring) {
                if (s.epi - s.hepi < (uint32_t)e.HR) h = e.hring + ((size_t)i * e.HR + (s.epi & (uint32_t)(e.HR - 1))) * EP_WORDS;
            } else {
                const uint32_t slot = atomicAdd(e.ep_count, 1u);
                if ((int)slot < e.ep_cap) h = e.ep_list + (size_t)slot * EP_WORDS;
            }
            if (h) {
                const uint32_t first = s.ep_first, nrec = s.rec - first;
                ((uint4*)h)[0] = make_uint4((uint32_t)(e.lane_base + i), s.epi, first, nrec);
                ((uint4*)h)[1] = make_uint4((uint32_t)s.steps,
                                            (uint32_t)win_type | ((uint32_t)(winner & 0xFF) << 8) |
                                                (s.flags << 16),
                                            s.w[0], s.w[1]);
                ((uint4*)h)[2] = make_uint4(s.w[2], s.w[3], s.w[4], s.w[5]);
                ((uint4*)h)[3] = make_uint4(s.w[6], 0u, 0u, 0u);
            } else {
                atomicOr(e.err_flags, BGX_ERRF_EPISODE_LIST);
            }
        }
        s.p = new_game(rng, s.w, s.d0, s.d1);
        s.steps = 0;
        s.flags = 0;
        s.epi = s.epi + 1;
        s.ep_first = s.rec;
    }
    if (lead) {
        store_packed(e.rows + (size_t)i * 8, s.w);
        if (rng.exhausted) atomicOr(e.err_flags, BGX_ERRF_DICE_EXHAUSTED);
    }
    s.ctr = rng.ctr;
}

// the phased engine's lane step: candidates at rows L + cand_off[i] + k, V in
// e.V; the lane's state from and back to memory (one thread)
BGX_DEV void step_lane(const EngineDev& e, int i, int action) {
    const int n_full = e.cand_cnt[i];
    const int n = n_full < e.max_legal ? n_full : e.max_legal;
    const int base = e.L + e.cand_off[i];
    const bool act = n > 0 && action >= 0;
    LaneState s;
    lane_load(e, i, s);
    uint32_t nb[8];
    load_packed(e.rows + (size_t)(base + (act ? action : 0)) * 8, nb);
    LaneRng rng;
    rng.key = lane_key(e.seed, (uint32_t)(e.lane_base + i));
    rng.ctr = s.ctr;
    rng.dt = lane_dice(e, i);
    lane_advance(e, i, s, rng, action, nb, e.V[i], act ? e.V[base + action] : 0.0f, n_full, true);
    lane_store(e, i, s);
}

// The lane's sampling uniform: Philox at its counter `ctr` (lane_advance
// advances the counter past it).
BGX_DEV float lane_uniform(const EngineDev& e, int i, uint64_t ctr) {
    return unit_from(philox(lane_key(e.seed, (uint32_t)(e.lane_base + i)), 0x5EED0000ull, ctr).x);
}
BGX_DEV float lane_uniform(const EngineDev& e, int i) { return lane_uniform(e, i, e.rng[i]); }

// Action choice over the scores x(0..m-1) (a functor; m >= 1) by one
// wavefront: softmax + inverse-CDF sample at uniform u (worker.py:137-143,
// torch Categorical), or with `greedy` the argmax, first maximum
// (play_versus_ai.py:188-195; the temperature does not change it).
template <typename X>
BGX_DEV int pick_action(X x, int m, bool greedy, float u) {
    const int l = lane_id();
    float mx = -INFINITY;
    for (int k = l; k < m; k += 64) mx = fmaxf(mx, x(k));
    mx = lane63f(wave_incl_maxf(mx));
    float sum = 0.0f;
    for (int k = l; k < m; k += 64) sum += __expf(x(k) - mx);
    sum = lane63f(wave_incl_scanf(sum));
    if (greedy) {
        float bv = -INFINITY;
        int bk = 0x7FFFFFFF;
        for (int k = l; k < m; k += 64) {
            const float xk = x(k);
            if (xk > bv) { bv = xk; bk = k; }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float ov = __shfl_xor(bv, off, 64);
            const int ok = __shfl_xor(bk, off, 64);
            if (ov > bv || (ov == bv && ok < bk)) { bv = ov; bk = ok; }
        }
        return bk;
    }
    int pick = m - 1;
    const float t = u * sum;
    float carry = 0.0f;
    for (int b = 0; b < m; b += 64) {
        const int k = b + l;
        const float p = wave_incl_scanf(k < m ? __expf(x(k) - mx) : 0.0f);   // inclusive scan over the wave
        const uint64_t hit = ballot(k < m && t < carry + p);
        if (hit) {
            pick = b + __ffsll((unsigned long long)hit) - 1;
            break;
        }
        carry += lane63f(p);
    }
    return pick;
}

// pick_action over one half-wave (lanes 32h .. 32h + 31 choose for one game
// lane, so a wavefront's two lanes choose side by side): softmax + inverse-CDF
// sample at uniform u, or the argmax with greedy, as pick_action, with 32-lane
// reductions. Every engine path uses this one, so the fused and phased
// engines sum the same terms in the same order (identical picks).
template <typename X>
BGX_DEV int pick_action_half(X x, int m, bool greedy, float u) {
    const int l = lane_id() & 31, hb = lane_id() & 32;
    if (m <= 64) {
        // up to two scores per lane, each read, divided and exponentiated once
        // (the same terms in the same order as the general loop below)
        const bool a0 = l < m, a1 = l + 32 < m;
        const float x0 = a0 ? x(l) : -INFINITY, x1 = a1 ? x(l + 32) : -INFINITY;
        float mx = fmaxf(fmaxf(-INFINITY, x0), x1);
        mx = half_last(half_incl_maxf(mx));
        if (greedy) {
            float bv = -INFINITY;
            int bk = 0x7FFFFFFF;
            if (a0 && x0 > bv) { bv = x0; bk = l; }
            if (a1 && x1 > bv) { bv = x1; bk = l + 32; }
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) {
                const float ov = __shfl_xor(bv, off, 64);
                const int ok = __shfl_xor(bk, off, 64);
                if (ov > bv || (ov == bv && ok < bk)) { bv = ov; bk = ok; }
            }
            return bk;
        }
        const float e0 = a0 ? __expf(x0 - mx) : 0.0f, e1 = a1 ? __expf(x1 - mx) : 0.0f;
        float s = 0.0f;
        if (a0) s += e0;
        if (a1) s += e1;
        const float ps = half_incl_scanf(s);
        const float sum = half_last(ps);
        const float t = u * sum;
        const float p0 = m <= 32 ? ps : half_incl_scanf(e0);   // s == e0 (exactly) when m <= 32
        const uint32_t h0 = (uint32_t)(ballot(a0 && t < 0.0f + p0) >> hb);
        if (h0) return __ffs(h0) - 1;
        const float carry = 0.0f + half_last(p0);
        if (m > 32) {
            const float p1 = half_incl_scanf(e1);
            const uint32_t h1 = (uint32_t)(ballot(a1 && t < carry + p1) >> hb);
            if (h1) return 32 + __ffs(h1) - 1;
        }
        return m - 1;
    }
    float mx = -INFINITY;
    for (int k = l; k < m; k += 32) mx = fmaxf(mx, x(k));
    mx = half_last(half_incl_maxf(mx));
    float sum = 0.0f;
    for (int k = l; k < m; k += 32) sum += __expf(x(k) - mx);
    sum = half_last(half_incl_scanf(sum));
    if (greedy) {
        float bv = -INFINITY;
        int bk = 0x7FFFFFFF;
        for (int k = l; k < m; k += 32) {
            const float xk = x(k);
            if (xk > bv) { bv = xk; bk = k; }
        }
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) {
            const float ov = __shfl_xor(bv, off, 64);
            const int ok = __shfl_xor(bk, off, 64);
            if (ov > bv || (ov == bv && ok < bk)) { bv = ov; bk = ok; }
        }
        return bk;
    }
    int pick = m - 1;
    const float t = u * sum;
    float carry = 0.0f;
    for (int b = 0; b < m; b += 32) {
        const int k = b + l;
        const float p = half_incl_scanf(k < m ? __expf(x(k) - mx) : 0.0f);
        const uint32_t hit = (uint32_t)(ballot(k < m && t < carry + p) >> hb);
        if (hit) {
            pick = b + __ffs(hit) - 1;
            break;
        }
        carry += half_last(p);
    }
    return pick;
}

}  // namespace bgx
