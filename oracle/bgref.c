/*
 * bgref.c — CPU restatement (TEST INFRASTRUCTURE ONLY; see bgref.h) of the
 * reference hot path. Every function cites the reference file:line it
 * follows. Written to be literal rather than fast: the doubles DFS, the
 * partial-record conditions, the shared unique-board set and the pass-2
 * skip are all reproduced as the reference writes them.
 */
#include "bgref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { P1 = 0, P2 = 1 };
enum { POS_BAR = 24, POS_OFF = 25 };
enum { ST_NORMAL = 1, ST_ON_BAR = 2, ST_BEAR_OFF = 3, ST_GAME_OVER = 4 };

typedef struct { uint8_t start, end, hit; } sub_t;
typedef struct { sub_t s[4]; int n; } full_t;

#define PTS(b, pl) ((b) + 24 * (pl))
#define BAR(b, pl) ((b)[48 + (pl)])
#define OFFC(b, pl) ((b)[50 + (pl)])

/* ---------------- conditions.py ---------------- */

/* check_for_win (conditions.py:137-149) */
static int check_for_win(const uint8_t* b, int pl) { return OFFC(b, pl) == 15; }
/* check_for_bar (conditions.py:122-134) */
static int check_for_bar(const uint8_t* b, int pl) { return BAR(b, pl) > 0; }

/* all_checkers_home (conditions.py:152-194) */
static int all_checkers_home(const uint8_t* b, int pl) {
    if (BAR(b, pl) > 0) return 0;
    int lo = pl == P2 ? 0 : 18, hi = pl == P2 ? 6 : 24;
    int total = 0;
    const uint8_t* p = PTS(b, pl);
    for (int idx = 0; idx < 24; ++idx) {
        int n = p[idx];
        if (n > 0) {
            if (idx >= lo && idx < hi) total += n;
            else return 0;
        }
    }
    return total + OFFC(b, pl) == 15;
}

/* compute_board_state (conditions.py:5-22) */
static int compute_board_state(const uint8_t* b, int pl) {
    if (check_for_win(b, pl)) return ST_GAME_OVER;
    if (check_for_bar(b, pl)) return ST_ON_BAR;
    if (all_checkers_home(b, pl)) return ST_BEAR_OFF;
    return ST_NORMAL;
}

/* valid_move (conditions.py:25-62) */
static int valid_move(int dest, int pl, const uint8_t* b) {
    if (dest >= 0 && dest < 24) return PTS(b, 1 - pl)[dest] >= 2 ? 0 : 1;
    if (dest == POS_OFF) return 1;
    return 0;
}
/* check_if_blot (conditions.py:65-89) */
static int check_if_blot(int idx, int pl, const uint8_t* b) {
    if (idx >= 0 && idx < 24) return PTS(b, 1 - pl)[idx] == 1;
    return 0;
}
/* is_valid_entry_at_index (conditions.py:92-119) */
static int is_valid_entry(int idx, int pl, const uint8_t* b) {
    if (idx >= 0 && idx < 24) return PTS(b, 1 - pl)[idx] >= 2 ? 0 : 1;
    return 0;
}

/* ---------------- get_moves_one_die.py ---------------- */

/* get_moves_normal (get_moves_one_die.py:40-83) */
static int moves_normal(const uint8_t* b, int d, int pl, sub_t* out) {
    int n = 0, dir = pl == P1 ? 1 : -1;
    const uint8_t* p = PTS(b, pl);
    for (int idx = 0; idx < 24; ++idx) {
        if (p[idx] > 0) {
            int dest = idx + d * dir;
            if (dest >= 0 && dest < 24 && valid_move(dest, pl, b)) {
                out[n].start = (uint8_t)idx;
                out[n].end = (uint8_t)dest;
                out[n].hit = (uint8_t)check_if_blot(dest, pl, b);
                ++n;
            }
        }
    }
    return n;
}

/* get_moves_bar (get_moves_one_die.py:86-130) */
static int moves_bar(const uint8_t* b, int d, int pl, sub_t* out) {
    if (BAR(b, pl) == 0) return 0;
    int dest, lo, hi;
    if (pl == P1) { dest = d - 1; lo = 0; hi = 6; }
    else { dest = 24 - d; lo = 18; hi = 24; }
    if (dest >= lo && dest < hi && is_valid_entry(dest, pl, b)) {
        out[0].start = POS_BAR;
        out[0].end = (uint8_t)dest;
        out[0].hit = (uint8_t)check_if_blot(dest, pl, b);
        return 1;
    }
    return 0;
}

/* get_moves_bear_off (get_moves_one_die.py:133-251) */
static int moves_bear_off(const uint8_t* b, int d, int pl, sub_t* out) {
    int n = 0, dir, last, h0;
    const uint8_t* p = PTS(b, pl);
    if (pl == P1) { h0 = 18; dir = 1; last = 18; }
    else { h0 = 0; dir = -1; last = 5; }
    /* 1. normal moves inside the home board, home indexes ascending */
    for (int k = 0; k < 6; ++k) {
        int idx = h0 + k;
        if (p[idx] > 0) {
            int dest = idx + d * dir;
            if (dest >= 0 && dest < 24 && valid_move(dest, pl, b)) {
                out[n].start = (uint8_t)idx;
                out[n].end = (uint8_t)dest;
                out[n].hit = (uint8_t)check_if_blot(dest, pl, b);
                ++n;
            }
        }
    }
    /* 2. farthest checker */
    if (pl == P1) {
        for (int idx = 18; idx < 24; ++idx) if (p[idx] > 0) { last = idx; break; }
    } else {
        for (int idx = 5; idx >= 0; --idx) if (p[idx] > 0) { last = idx; break; }
    }
    /* 3. bear-off moves */
    if (pl == P1) {
        if (last + d * dir >= 24) {
            out[n].start = (uint8_t)last; out[n].end = POS_OFF; out[n].hit = 0; ++n;
        }
        int ps = 24 - d;
        if (ps != last && ps >= 18 && ps < 24 && p[ps] > 0) {
            out[n].start = (uint8_t)ps; out[n].end = POS_OFF; out[n].hit = 0; ++n;
        }
    } else {
        if (last + d * dir < 0) {
            out[n].start = (uint8_t)last; out[n].end = POS_OFF; out[n].hit = 0; ++n;
        }
        int ps = d - 1;
        if (ps != last && ps >= 0 && ps < 6 && p[ps] > 0) {
            out[n].start = (uint8_t)ps; out[n].end = POS_OFF; out[n].hit = 0; ++n;
        }
    }
    return n;
}

/* get_moves_with_one_die (get_moves_one_die.py:13-37) */
static int moves_one_die(const uint8_t* b, int d, int pl, sub_t* out) {
    switch (compute_board_state(b, pl)) {
        case ST_NORMAL: return moves_normal(b, d, pl, out);
        case ST_ON_BAR: return moves_bar(b, d, pl, out);
        case ST_BEAR_OFF: return moves_bear_off(b, d, pl, out);
        default: return 0;
    }
}

/* ImmutableBoard.move_checker (immutable_board.py:183-258): returns 0 and
 * leaves `out` = `b` on the reference's "invalid, return self" branches. */
static void move_checker(const uint8_t* b, int pl, sub_t m, uint8_t* out) {
    uint8_t t[52];
    memcpy(t, b, 52);
    int op = 1 - pl;
    if (m.start == POS_BAR) {
        if (BAR(t, pl) <= 0) { memcpy(out, b, 52); return; }
        BAR(t, pl) -= 1;
    } else {
        if (PTS(t, pl)[m.start] <= 0) { memcpy(out, b, 52); return; }
        PTS(t, pl)[m.start] -= 1;
    }
    if (m.hit) {
        if (PTS(t, op)[m.end] == 1) {
            PTS(t, op)[m.end] -= 1;
            BAR(t, op) += 1;
        } else { memcpy(out, b, 52); return; }
    }
    if (m.end == POS_OFF) OFFC(t, pl) += 1;
    else PTS(t, pl)[m.end] += 1;
    memcpy(out, t, 52);
}

/* execute_full_move_on_board_copy (env_helper.py:27-91): no validity checks */
static void execute_full_move(const uint8_t* b, int pl, const full_t* fm, uint8_t* out) {
    memcpy(out, b, 52);
    int op = 1 - pl;
    for (int i = 0; i < fm->n; ++i) {
        sub_t s = fm->s[i];
        if (s.start == POS_BAR) BAR(out, pl) -= 1;
        else PTS(out, pl)[s.start] -= 1;
        if (s.hit) { PTS(out, op)[s.end] -= 1; BAR(out, op) += 1; }
        if (s.end == POS_OFF) OFFC(out, pl) += 1;
        else PTS(out, pl)[s.end] += 1;
    }
}

/* ---------------- unique board set (handle_move_types.py:196-221) -------- */

typedef struct {
    uint8_t* keys;   /* cap * 52 */
    uint8_t* used;
    int cap;
    int count;
} board_set;

static uint64_t hash52(const uint8_t* b) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 52; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static void set_init(board_set* s, int cap) {
    s->cap = cap;
    s->count = 0;
    s->keys = (uint8_t*)malloc((size_t)cap * 52);
    s->used = (uint8_t*)calloc((size_t)cap, 1);
}
static void set_free(board_set* s) { free(s->keys); free(s->used); }

static void set_grow(board_set* s);
/* returns 1 if inserted (was absent) */
static int set_add(board_set* s, const uint8_t* b) {
    if (2 * (s->count + 1) > s->cap) set_grow(s);
    uint64_t h = hash52(b) & (uint64_t)(s->cap - 1);
    for (;;) {
        if (!s->used[h]) {
            s->used[h] = 1;
            memcpy(s->keys + h * 52, b, 52);
            s->count++;
            return 1;
        }
        if (memcmp(s->keys + h * 52, b, 52) == 0) return 0;
        h = (h + 1) & (uint64_t)(s->cap - 1);
    }
}
static void set_grow(board_set* s) {
    board_set n;
    set_init(&n, s->cap * 2);
    for (int i = 0; i < s->cap; ++i)
        if (s->used[i]) set_add(&n, s->keys + (size_t)i * 52);
    set_free(s);
    *s = n;
}

typedef struct {
    full_t* moves;
    int n, cap;
    board_set set;
} move_list;

static void ml_init(move_list* ml) {
    ml->cap = 256;
    ml->n = 0;
    ml->moves = (full_t*)malloc(sizeof(full_t) * ml->cap);
    set_init(&ml->set, 1024);
}

/* add_unique_board (handle_move_types.py:196-221) */
static void add_unique_board(move_list* ml, const uint8_t* board, const sub_t* seq, int n) {
    if (!set_add(&ml->set, board)) return;
    if (ml->n == ml->cap) {
        ml->cap *= 2;
        ml->moves = (full_t*)realloc(ml->moves, sizeof(full_t) * ml->cap);
    }
    full_t* fm = &ml->moves[ml->n++];
    fm->n = n;
    for (int i = 0; i < n; ++i) fm->s[i] = seq[i];
}

/* handle_non_doubles (handle_move_types.py:7-81) */
static void handle_non_doubles(const uint8_t* board, int r0, int r1, move_list* ml,
                               int pl, int reverse) {
    int d_first = reverse ? r1 : r0, d_second = reverse ? r0 : r1;
    sub_t first[16], second[16];
    int nf = moves_one_die(board, d_first, pl, first);
    int two = 0;
    uint8_t b1[52], b2[52];
    for (int i = 0; i < nf; ++i) {
        move_checker(board, pl, first[i], b1);
        int ns = moves_one_die(b1, d_second, pl, second);
        if (ns) {
            two = 1;
            for (int j = 0; j < ns; ++j) {
                move_checker(b1, pl, second[j], b2);
                sub_t seq[2] = {first[i], second[j]};
                add_unique_board(ml, b2, seq, 2);
            }
        }
    }
    if (!two) {
        for (int i = 0; i < nf; ++i) {
            move_checker(board, pl, first[i], b1);
            add_unique_board(ml, b1, &first[i], 1);
        }
    }
}

/* handle_doubles (handle_move_types.py:84-193) */
static void handle_doubles(const uint8_t* board, int d, move_list* ml, int pl) {
    sub_t m1[16], m2[16], m3[16], m4[16];
    uint8_t b1[52], b2[52], b3[52], b4[52];
    int n1 = moves_one_die(board, d, pl, m1);
    int full4 = 0;
    for (int i = 0; i < n1; ++i) {
        move_checker(board, pl, m1[i], b1);
        int n2 = moves_one_die(b1, d, pl, m2);
        if (!n2 && n1 == 1 && !full4) {
            sub_t seq[1] = {m1[i]};
            add_unique_board(ml, b1, seq, 1);
        }
        for (int j = 0; j < n2; ++j) {
            move_checker(b1, pl, m2[j], b2);
            int n3 = moves_one_die(b2, d, pl, m3);
            if (!n3 && n2 == 1 && !full4) {
                sub_t seq[2] = {m1[i], m2[j]};
                add_unique_board(ml, b2, seq, 2);
            }
            for (int k = 0; k < n3; ++k) {
                move_checker(b2, pl, m3[k], b3);
                int n4 = moves_one_die(b3, d, pl, m4);
                if (!n4 && n3 == 1 && !full4) {
                    sub_t seq[3] = {m1[i], m2[j], m3[k]};
                    add_unique_board(ml, b3, seq, 3);
                }
                for (int l = 0; l < n4; ++l) {
                    move_checker(b3, pl, m4[l], b4);
                    sub_t seq[4] = {m1[i], m2[j], m3[k], m4[l]};
                    add_unique_board(ml, b4, seq, 4);
                    full4 = 1;
                }
            }
        }
    }
}

/* get_all_possible_moves (generate_all_moves.py:7-66) + filter (69-90).
 * Returns count; fills *out (malloc'd, caller frees). */
static int all_moves(const uint8_t* board, int pl, int d0, int d1, full_t** out) {
    move_list ml;
    ml_init(&ml);
    if (d0 != d1) {
        int hi = d0 > d1 ? d0 : d1, lo = d0 > d1 ? d1 : d0;
        handle_non_doubles(board, hi, lo, &ml, pl, 0);
        if (ml.n == 0 || !(ml.n == 1 && ml.moves[0].n == 1))
            handle_non_doubles(board, hi, lo, &ml, pl, 1);
    } else {
        handle_doubles(board, d0, &ml, pl);
    }
    int mx = 0;
    for (int i = 0; i < ml.n; ++i) if (ml.moves[i].n > mx) mx = ml.moves[i].n;
    int k = 0;
    for (int i = 0; i < ml.n; ++i) if (ml.moves[i].n == mx) ml.moves[k++] = ml.moves[i];
    *out = ml.moves;
    ml.moves = NULL;
    set_free(&ml.set);
    return k;
}

int bgref_movegen_full(const uint8_t* board, int player, int d0, int d1,
                       uint8_t* out_boards, int cap, uint8_t* out_nsub,
                       uint8_t* out_sub) {
    full_t* fm;
    int n = all_moves(board, player, d0, d1, &fm);
    int w = n < cap ? n : cap;
    for (int i = 0; i < w; ++i) {
        if (out_boards) execute_full_move(board, player, &fm[i], out_boards + (size_t)i * 52);
        if (out_nsub) out_nsub[i] = (uint8_t)fm[i].n;
        if (out_sub) {
            uint8_t* s = out_sub + (size_t)i * 12;
            memset(s, 0, 12);
            for (int j = 0; j < fm[i].n; ++j) {
                s[3 * j] = fm[i].s[j].start;
                s[3 * j + 1] = fm[i].s[j].end;
                s[3 * j + 2] = fm[i].s[j].hit;
            }
        }
    }
    free(fm);
    return n;
}

int bgref_movegen(const uint8_t* board, int player, int d0, int d1,
                  uint8_t* out_boards, int cap, uint8_t* out_nsub) {
    return bgref_movegen_full(board, player, d0, d1, out_boards, cap, out_nsub, NULL);
}

/* ---------------- encoders ---------------- */

static float point_feat(int n, int c) {
    switch (c) {
        case 0: return n >= 1 ? 1.0f : 0.0f;
        case 1: return n >= 2 ? 1.0f : 0.0f;
        case 2: return n >= 3 ? 1.0f : 0.0f;
        default: return n > 3 ? (float)(n - 3) / 2.0f : 0.0f;
    }
}

void bgref_encode(const uint8_t* b, int player, int layout, float* f) {
    if (layout == 0) {
        /* get_board_features (immutable_board.py:86-128): [P1 pts | P2 pts | bar1 off1 bar2 off2 | flags] */
        for (int pl = 0; pl < 2; ++pl)
            for (int i = 0; i < 24; ++i)
                for (int c = 0; c < 4; ++c) f[96 * pl + 4 * i + c] = point_feat(PTS(b, pl)[i], c);
        f[192] = (float)(BAR(b, P1) / 2.0);
        f[193] = (float)(OFFC(b, P1) / 15.0);
        f[194] = (float)(BAR(b, P2) / 2.0);
        f[195] = (float)(OFFC(b, P2) / 15.0);
    } else {
        /* compute_features (generate_board_tensor.py:98-140): per player pts, bar, off */
        int k = 0;
        for (int pl = 0; pl < 2; ++pl) {
            for (int i = 0; i < 24; ++i)
                for (int c = 0; c < 4; ++c) f[k++] = point_feat(PTS(b, pl)[i], c);
            f[k++] = (float)(BAR(b, pl) / 2.0);
            f[k++] = (float)(OFFC(b, pl) / 15.0);
        }
    }
    f[196] = player == P1 ? 1.0f : 0.0f;
    f[197] = player == P2 ? 1.0f : 0.0f;
}

/* ---------------- MLP (policy_network.py:53-70) ---------------- */

void bgref_value(const float* W1, const float* b1, const float* w2, const float* b2,
                 const float* x, int n, double* out) {
    /* fp64 sums in feature order over the nonzero features only: a zero
     * feature adds an exact (+-)0 to the running sum, so skipping it leaves
     * every h bit-identical to the dense loop (a live row has ~28 nonzeros of
     * 198, which makes the 2-ply checks ~7x cheaper) */
    int nz[BGREF_NFEAT];
    for (int r = 0; r < n; ++r) {
        const float* xr = x + (size_t)r * BGREF_NFEAT;
        int m = 0;
        for (int k = 0; k < BGREF_NFEAT; ++k)
            if (xr[k] != 0.0f) nz[m++] = k;
        double v = b2[0];
        for (int j = 0; j < BGREF_HIDDEN; ++j) {
            double h = b1[j];
            const float* w = W1 + (size_t)j * BGREF_NFEAT;
            for (int q = 0; q < m; ++q) h += (double)w[nz[q]] * (double)xr[nz[q]];
            v += (double)w2[j] * (1.0 / (1.0 + exp(-h)));
        }
        out[r] = v;
    }
}

void bgref_value_f32(const float* W1, const float* b1, const float* w2, const float* b2,
                     const float* x, int n, float* out) {
    for (int r = 0; r < n; ++r) {
        const float* xr = x + (size_t)r * BGREF_NFEAT;
        float v = 0.0f;
        for (int j = 0; j < BGREF_HIDDEN; ++j) {
            float h = 0.0f;
            const float* w = W1 + (size_t)j * BGREF_NFEAT;
            for (int k = 0; k < BGREF_NFEAT; ++k) h += w[k] * xr[k];
            h += b1[j];
            v += w2[j] * (1.0f / (1.0f + expf(-h)));
        }
        out[r] = v + b2[0];
    }
}

/* ---------------- env_helper.py reward predicates ---------------- */

/* check_game_over (env_helper.py:113-117) */
int bgref_check_game_over(const uint8_t* b, int pl) { return OFFC(b, pl) >= 15; }
/* check_for_gammon (env_helper.py:120-127) */
int bgref_check_for_gammon(const uint8_t* b, int pl) { return OFFC(b, 1 - pl) == 0; }
/* check_for_backgammon (env_helper.py:130-163) */
int bgref_check_for_backgammon(const uint8_t* b, int pl) {
    int op = 1 - pl;
    if (OFFC(b, op) > 0) return 0;
    int lo = pl == P1 ? 18 : 0;
    for (int idx = lo; idx < lo + 6; ++idx) if (PTS(b, op)[idx] > 0) return 1;
    if (BAR(b, op) > 0) return 1;
    return 0;
}
/* made_at_least_five_prime (env_helper.py:167-215) */
int bgref_made_at_least_five_prime(const uint8_t* b, int pl) {
    const uint8_t* me = PTS(b, pl);
    const uint8_t* op = PTS(b, 1 - pl);
    int len = 0;
    for (int t = 0; t < 24; ++t) {
        int idx = pl == P1 ? t : 23 - t;
        if (me[idx] >= 2) len++;
        else len = 0;
        if (len >= 5) {
            int lo, hi;
            if (pl == P1) { lo = idx + 1; hi = 24; }
            else { lo = 0; hi = idx; }
            for (int i = lo; i < hi; ++i) if (op[i] > 0) return 1;
        }
    }
    return 0;
}
/* is_closed_out (env_helper.py:218-242) */
int bgref_is_closed_out(const uint8_t* b, int pl) {
    int op = 1 - pl;
    if (BAR(b, op) == 0) return 0;
    int lo = pl == P1 ? 18 : 0;
    for (int idx = lo; idx < lo + 6; ++idx) if (PTS(b, pl)[idx] < 2) return 0;
    return 1;
}

/* ---------------- 2-ply (two_ply.py:10-35, 93-150) ---------------- */

static const int DICE_ROLLS[21][2] = {
    {1, 1}, {1, 2}, {1, 3}, {1, 4}, {1, 5}, {1, 6}, {2, 2}, {2, 3}, {2, 4}, {2, 5}, {2, 6},
    {3, 3}, {3, 4}, {3, 5}, {3, 6}, {4, 4}, {4, 5}, {4, 6}, {5, 5}, {5, 6}, {6, 6}};
static const int COUNTS[21] = {1, 2, 2, 2, 2, 2, 1, 2, 2, 2, 2, 1, 2, 2, 2, 1, 2, 2, 1, 2, 1};

static int cmp_desc(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return (x < y) - (x > y);
}

double bgref_two_ply_response(const uint8_t* board, int opp, const float* W1,
                              const float* b1, const float* w2, const float* b2) {
    double total = 0.0;
    for (int r = 0; r < 21; ++r) {
        full_t* fm;
        int n = all_moves(board, opp, DICE_ROLLS[r][0], DICE_ROLLS[r][1], &fm);
        if (n > 0) {
            double* v = (double*)malloc(sizeof(double) * n);
            float x[BGREF_NFEAT];
            uint8_t nb[52];
            for (int i = 0; i < n; ++i) {
                execute_full_move(board, opp, &fm[i], nb);
                bgref_encode(nb, opp, 0, x);
                bgref_value(W1, b1, w2, b2, x, 1, &v[i]);
            }
            qsort(v, n, sizeof(double), cmp_desc);
            int k = n < 5 ? n : 5;
            double s = 0.0;
            for (int i = 0; i < k; ++i) s += v[i];
            total += (s / k) * ((double)COUNTS[r] / 36.0);
            free(v);
        }
        free(fm);
    }
    return total;
}

/* ---------------- environment (backgammon_env.py) ---------------- */

static const uint8_t INITIAL[52] = {
    /* P1 (immutable_board.py:34-37): 0:2, 11:5, 16:3, 18:5 */
    2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 5, 0, 0, 0, 0, 3, 0, 5, 0, 0, 0, 0, 0,
    /* P2 (immutable_board.py:40-43): 23:2, 12:5, 7:3, 5:5 */
    0, 0, 0, 0, 0, 5, 0, 3, 0, 0, 0, 0, 5, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2,
    0, 0, 0, 0};

static int env_die(bgref_env* e) {
    if (e->dice_pos >= e->n_dice) return -1;
    return e->dice[e->dice_pos++];
}
/* roll_dice (backgammon_env.py:310-311) */
static int env_roll(bgref_env* e) {
    int a = env_die(e), b = env_die(e);
    if (a < 0 || b < 0) return -1;
    e->roll[0] = a;
    e->roll[1] = b;
    return 0;
}
/* update_legal_moves + truncate (backgammon_env.py:223-272) */
static void env_update_legal(bgref_env* e) {
    full_t* fm;
    int n = all_moves(e->board, e->current_player, e->roll[0], e->roll[1], &fm);
    e->full_moves = n;
    int w = n < e->max_legal_moves ? n : e->max_legal_moves;
    for (int i = 0; i < w; ++i)
        execute_full_move(e->board, e->current_player, &fm[i], e->legal_boards + (size_t)i * 52);
    e->num_moves = w;
    free(fm);
}

int bgref_env_init(bgref_env* e, uint8_t* legal_boards, int max_legal_moves,
                   const int* dice, int n_dice) {
    memset(e, 0, sizeof(*e));
    memcpy(e->board, INITIAL, 52);
    e->legal_boards = legal_boards;
    e->max_legal_moves = max_legal_moves;
    e->dice = dice;
    e->n_dice = n_dice;
    return 0;
}

/* reset (backgammon_env.py:92-128) */
int bgref_env_reset(bgref_env* e) {
    memcpy(e->board, INITIAL, 52);
    e->game_over = 0;
    if (env_roll(e)) return -1;
    while (e->roll[0] == e->roll[1]) if (env_roll(e)) return -1;
    e->current_player = e->roll[0] < e->roll[1] ? P2 : P1;
    if (env_roll(e)) return -1;
    while (e->roll[0] == e->roll[1]) if (env_roll(e)) return -1;
    env_update_legal(e);
    e->close_out_given[0] = e->close_out_given[1] = 0;
    e->prime_given[0] = e->prime_given[1] = 0;
    return 0;
}

/* step (backgammon_env.py:130-221) */
int bgref_env_step(bgref_env* e, int action, bgref_step_result* r) {
    memset(r, 0, sizeof(*r));
    r->info_current_player = e->current_player;
    r->winner = -1;
    if (e->game_over) { r->done = 1; r->kind = 3; return 0; }
    if (e->num_moves == 0) {
        r->kind = 1;
        e->current_player = 1 - e->current_player;
        if (env_roll(e)) return -1;
        env_update_legal(e);
        return 0;
    }
    if (action < 0 || action >= e->num_moves) { r->reward = -1.0f; r->kind = 2; return 0; }
    memcpy(e->board, e->legal_boards + (size_t)action * 52, 52);
    float reward = 0.0f;
    int pl = e->current_player;
    if (bgref_check_game_over(e->board, pl)) {
        if (bgref_check_for_backgammon(e->board, pl)) { reward = 2.5f; r->win_type = 3; }
        else if (bgref_check_for_gammon(e->board, pl)) { reward = 2.0f; r->win_type = 2; }
        else { reward = 1.0f; r->win_type = 1; }
        r->winner = pl;
        e->game_over = 1;
        r->done = 1;
    } else {
        if (bgref_is_closed_out(e->board, pl) && !e->close_out_given[pl]) {
            reward += 0.30f;
            e->close_out_given[pl] = 1;
            r->close_out_reward = 1;
        }
        if (bgref_made_at_least_five_prime(e->board, pl) && !e->prime_given[pl]) {
            reward += 0.20f;
            e->prime_given[pl] = 1;
            r->prime_reward = 1;
        }
        e->current_player = 1 - pl;
        if (env_roll(e)) return -1;
        env_update_legal(e);
    }
    r->reward = reward;
    return 0;
}

/* ---------------- Philox4x32-10 ---------------- */

void bgref_philox4x32(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo, uint32_t out[4]) {
    uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
    uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* ---------------- CPU self-play port (worker.py:78-174) ---------------- */

typedef struct {
    const float *W1, *b1, *w2, *b2;
    float temperature;
    uint64_t seed;
    int tid;
    double seconds;
    long long steps, decisions, episodes;
    int ply;          /* 1: softmax(V/T) over every candidate (worker.py:137-143);
                         2: two_ply.py:44-90 scoring of the top-4 by V, softmax over the four */
    long long warmup; /* untimed env steps first (a 300-step warm-up): whole games at ply 1; at
                         ply 2 1-ply decisions, ending mid-game so the 2-ply window starts in the mix */
    double elapsed;   /* the thread's timed window */
} sp_arg;

/* compute_weighted_opponent_response (two_ply.py:93-150), exact mode, in
 * fp32 batches (the CPU port's arithmetic, like bgref_value_f32) */
static double two_ply_response_f32(const uint8_t* board, int opp, const sp_arg* a, float* x, float* v) {
    double total = 0.0;
    for (int r = 0; r < 21; ++r) {
        full_t* fm;
        int n = all_moves(board, opp, DICE_ROLLS[r][0], DICE_ROLLS[r][1], &fm);
        if (n > 0) {
            uint8_t nb[52];
            int done = 0;
            double top[5];
            int nt = 0;
            while (done < n) {   /* batches of up to 500 replies */
                const int b = n - done < 500 ? n - done : 500;
                for (int i = 0; i < b; ++i) {
                    execute_full_move(board, opp, &fm[done + i], nb);
                    bgref_encode(nb, opp, 0, x + (size_t)i * BGREF_NFEAT);
                }
                bgref_value_f32(a->W1, a->b1, a->w2, a->b2, x, b, v);
                for (int i = 0; i < b; ++i) {   /* running top 5, descending */
                    double y = v[i];
                    int k = nt < 5 ? nt++ : 5;
                    if (k == 5 && y <= top[4]) continue;
                    if (k == 5) k = 4;
                    while (k > 0 && top[k - 1] < y) { top[k] = top[k - 1]; --k; }
                    top[k] = y;
                }
                done += b;
            }
            double s = 0.0;
            for (int i = 0; i < nt; ++i) s += top[i];
            total += (s / nt) * ((double)COUNTS[r] / 36.0);
        }
        free(fm);
    }
    return total;
}

typedef struct {
    uint64_t key;
    uint64_t ctr;
    uint32_t buf[4];
    int pos;
} sp_rng;

static uint32_t rng_u32(sp_rng* r) {
    if (r->pos == 4) { bgref_philox4x32(r->key, 0, r->ctr++, r->buf); r->pos = 0; }
    return r->buf[r->pos++];
}
static int rng_die(sp_rng* r) { return 1 + (int)(((uint64_t)rng_u32(r) * 6u) >> 32); }

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void sp_roll(uint8_t roll[2], sp_rng* r) { roll[0] = (uint8_t)rng_die(r); roll[1] = (uint8_t)rng_die(r); }

static void* sp_thread(void* p) {
    sp_arg* a = (sp_arg*)p;
    sp_rng rng = {a->seed * 0x9E3779B97F4A7C15ull + (uint64_t)a->tid, 0, {0}, 4};
    uint8_t* legal = (uint8_t*)malloc(500 * 52);
    float* x = (float*)malloc(sizeof(float) * 501 * BGREF_NFEAT);
    float* v = (float*)malloc(sizeof(float) * 501);
    double* pr = (double*)malloc(sizeof(double) * 501);
    float* x2 = (float*)malloc(sizeof(float) * 500 * BGREF_NFEAT);
    float* v2 = (float*)malloc(sizeof(float) * 500);
    double t0 = now_s();
    long long steps = 0, dec = 0, eps = 0;
    int warm = a->warmup > 0;
    while (warm || now_s() - t0 < a->seconds) {
        /* reset (backgammon_env.py:92-128) */
        uint8_t board[52], roll[2];
        memcpy(board, INITIAL, 52);
        int pl;
        do sp_roll(roll, &rng); while (roll[0] == roll[1]);
        pl = roll[0] < roll[1] ? P2 : P1;
        do sp_roll(roll, &rng); while (roll[0] == roll[1]);
        int co[2] = {0, 0}, pg[2] = {0, 0};
        int done = 0, step = 0;
        while (!done && step < 300) {
            /* 2-ply: the warm-up plays 1-ply decisions (cheap) and ends mid-game,
               so the timed 2-ply window starts from the self-play position mix */
            if (warm && a->ply == 2 && steps + step >= a->warmup) {
                warm = 0;
                steps = -step;   /* += step at the game's end: the steps after the switch */
                dec = eps = 0;
                t0 = now_s();
            }
            full_t* fm;
            int n = all_moves(board, pl, roll[0], roll[1], &fm);
            if (n > 500) n = 500;
            if (n == 0) {
                free(fm);
                pl = 1 - pl;
                sp_roll(roll, &rng);
                ++step;
                continue;
            }
            bgref_encode(board, pl, 0, x);
            for (int i = 0; i < n; ++i) {
                execute_full_move(board, pl, &fm[i], legal + (size_t)i * 52);
                bgref_encode(legal + (size_t)i * 52, pl, 0, x + (size_t)(i + 1) * BGREF_NFEAT);
            }
            free(fm);
            bgref_value_f32(a->W1, a->b1, a->w2, a->b2, x, n + 1, v);
            /* scores: 1-ply V, or (2-ply, >= 4 moves) alpha*V - beta*W of the top 4 by V */
            int cand[500], m = n;
            double sc[500];
            for (int i = 0; i < n; ++i) { cand[i] = i; sc[i] = v[i + 1]; }
            if (a->ply == 2 && n >= 4 && !warm) {
                for (int c = 0; c < 4; ++c) {   /* top-4 by V, ties to the lower index */
                    int best = c;
                    for (int i = c + 1; i < n; ++i)
                        if (v[cand[i] + 1] > v[cand[best] + 1] ||
                            (v[cand[i] + 1] == v[cand[best] + 1] && cand[i] < cand[best])) best = i;
                    int t = cand[c]; cand[c] = cand[best]; cand[best] = t;
                }
                m = 4;
                for (int c = 0; c < 4; ++c)
                    sc[c] = 1.0 * v[cand[c] + 1] -
                            0.9 * two_ply_response_f32(legal + (size_t)cand[c] * 52, 1 - pl, a, x2, v2);
            }
            double mx = -1e300, s = 0.0;
            for (int i = 0; i < m; ++i) if (sc[i] / a->temperature > mx) mx = sc[i] / a->temperature;
            for (int i = 0; i < m; ++i) { pr[i] = exp(sc[i] / a->temperature - mx); s += pr[i]; }
            double u = (rng_u32(&rng) >> 8) * (1.0 / 16777216.0) * s;
            int act = m - 1;
            for (int i = 0; i < m; ++i) { u -= pr[i]; if (u < 0) { act = i; break; } }
            act = cand[act];
            memcpy(board, legal + (size_t)act * 52, 52);
            if (bgref_check_game_over(board, pl)) {
                (void)bgref_check_for_backgammon(board, pl);
                done = 1;
            } else {
                if (bgref_is_closed_out(board, pl) && !co[pl]) co[pl] = 1;
                if (bgref_made_at_least_five_prime(board, pl) && !pg[pl]) pg[pl] = 1;
                pl = 1 - pl;
                sp_roll(roll, &rng);
            }
            ++dec;
            ++step;
        }
        steps += step;
        ++eps;
        if (warm && steps >= a->warmup) {   /* the warm-up ends at a game boundary: start the clock */
            warm = 0;
            steps = dec = eps = 0;
            t0 = now_s();
        }
    }
    a->elapsed = now_s() - t0;
    a->steps = steps;
    a->decisions = dec;
    a->episodes = eps;
    free(legal); free(x); free(v); free(pr); free(x2); free(v2);
    return NULL;
}

long long bgref_selfplay_bench(const float* W1, const float* b1, const float* w2,
                               const float* b2, float temperature, uint64_t seed,
                               int n_threads, double seconds, long long* decisions,
                               long long* episodes, double* elapsed) {
    return bgref_selfplay_bench_ply(W1, b1, w2, b2, temperature, seed, n_threads, seconds, 1,
                                    decisions, episodes, elapsed);
}

long long bgref_selfplay_bench_ply(const float* W1, const float* b1, const float* w2,
                                   const float* b2, float temperature, uint64_t seed,
                                   int n_threads, double seconds, int ply, long long* decisions,
                                   long long* episodes, double* elapsed) {
    return bgref_selfplay_bench_warm(W1, b1, w2, b2, temperature, seed, n_threads, seconds, ply, 0,
                                     decisions, episodes, elapsed);
}

long long bgref_selfplay_bench_warm(const float* W1, const float* b1, const float* w2,
                                    const float* b2, float temperature, uint64_t seed,
                                    int n_threads, double seconds, int ply, long long warmup,
                                    long long* decisions, long long* episodes, double* elapsed) {
    if (n_threads < 1) n_threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
    sp_arg* args = (sp_arg*)calloc(n_threads, sizeof(sp_arg));
    for (int i = 0; i < n_threads; ++i) {
        args[i] = (sp_arg){W1, b1, w2, b2, temperature, seed, i, seconds, 0, 0, 0, ply, warmup, 0.0};
        pthread_create(&th[i], NULL, sp_thread, &args[i]);
    }
    long long s = 0, d = 0, e = 0;
    double el = 0.0;   /* the longest thread window (each starts after its own warm-up) */
    for (int i = 0; i < n_threads; ++i) {
        pthread_join(th[i], NULL);
        s += args[i].steps; d += args[i].decisions; e += args[i].episodes;
        if (args[i].elapsed > el) el = args[i].elapsed;
    }
    if (elapsed) *elapsed = el;
    if (decisions) *decisions = d;
    if (episodes) *episodes = e;
    free(th); free(args);
    return s;
}
