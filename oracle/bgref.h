/*
 * bgref.h — CPU restatement (TEST INFRASTRUCTURE ONLY) of the reference
 * backgammon self-play hot path of Nick-qsv/MLP-PPO-2PLY-MULTI.
 *
 * ORACLE HEADER: this library is the parity checker. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (libbgx.so, the bgx Python package) never links,
 * imports or calls anything under oracle/.
 *
 * Parity pinning: every function is checked against golden vectors that
 * tools/gen_golden.py produced by importing the reference Python package
 * in the build container (tests/golden/, see tests/test_oracle_golden.py).
 *
 * Board layout ("u8[52]", the reference's ImmutableBoard fields in order):
 *   b[0..23]  positions_0 (PLAYER1 checkers per point)
 *   b[24..47] positions_1 (PLAYER2 checkers per point)
 *   b[48..49] bar[PLAYER1], bar[PLAYER2]
 *   b[50..51] borne_off[PLAYER1], borne_off[PLAYER2]
 *   (src/backgammon/board/immutable_board.py:16-24)
 */
#ifndef BGREF_H
#define BGREF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BGREF_BOARD_BYTES 52
#define BGREF_NFEAT 198
#define BGREF_HIDDEN 128
#define BGREF_MAX_RESULTS 8192

/* get_all_possible_moves (src/backgammon/moves/generate_all_moves.py:7-66).
 * Writes min(count, cap) result boards (execute_full_move_on_board_copy of
 * each FullMove, env_helper.py:27-91) in the reference's order to out_boards
 * (cap x 52 bytes) and, if out_nsub != NULL, the sub-move count of each.
 * Returns the full count (may exceed cap). */
int bgref_movegen(const uint8_t* board, int player, int d0, int d1,
                  uint8_t* out_boards, int cap, uint8_t* out_nsub);

/* Same, also returning each FullMove's sub-moves: out_sub[cap][4][3]
 * (start, end, hits_blot), start/end as Position ints (BAR=24, BEAR_OFF=25). */
int bgref_movegen_full(const uint8_t* board, int player, int d0, int d1,
                       uint8_t* out_boards, int cap, uint8_t* out_nsub,
                       uint8_t* out_sub);

/* ImmutableBoard.get_board_features (immutable_board.py:86-128), layout 0
 * (LIVE), or generate_board_tensor.compute_features (generate_board_tensor.py:
 * 98-140), layout 1 (interleaved, dead in the reference). */
void bgref_encode(const uint8_t* board, int player, int layout, float* out198);

/* BackgammonPolicyNetwork.forward (src/agents/policy_network.py:53-70):
 * V = w2 . sigmoid(W1 x + b1) + b2, W1 row-major [128][198].
 * Computed in double (the 1e-5 parity reference). */
void bgref_value(const float* W1, const float* b1, const float* w2,
                 const float* b2, const float* x, int n, double* out);
/* fp32 variant (same op order as a naive fp32 GEMV) — used by the CPU port. */
void bgref_value_f32(const float* W1, const float* b1, const float* w2,
                     const float* b2, const float* x, int n, float* out);

/* env_helper.py reward predicates (env_helper.py:113-242). */
int bgref_check_game_over(const uint8_t* board, int player);
int bgref_check_for_gammon(const uint8_t* board, int player);
int bgref_check_for_backgammon(const uint8_t* board, int player);
int bgref_made_at_least_five_prime(const uint8_t* board, int player);
int bgref_is_closed_out(const uint8_t* board, int player);

/* compute_weighted_opponent_response (src/multi/two_ply.py:93-150) in exact
 * mode (no random.sample for 1-1/2-2/3-3). */
double bgref_two_ply_response(const uint8_t* board, int opponent,
                              const float* W1, const float* b1,
                              const float* w2, const float* b2);

/* ---- Environment (src/environments/backgammon_env.py) -------------------- */
typedef struct bgref_env {
    uint8_t board[52];
    int current_player;
    int game_over;
    int roll[2];
    int close_out_given[2];
    int prime_given[2];
    int num_moves;          /* after truncation to max_legal_moves */
    int full_moves;         /* before truncation */
    int max_legal_moves;    /* 500 (backgammon_env.py:35) */
    uint8_t* legal_boards;  /* [max_legal_moves][52], owned by caller */
    /* dice source: sequence of single-die draws (np.random.randint(1,7)) */
    const int* dice;
    int n_dice;
    int dice_pos;
} bgref_env;

/* Step result (backgammon_env.py:130-221). win_type: 0 none, 1 regular,
 * 2 gammon, 3 backgammon. kind: 0 move, 1 pass, 2 invalid, 3 already over. */
typedef struct bgref_step_result {
    float reward;
    int done;
    int info_current_player;
    int winner;
    int win_type;
    int close_out_reward;
    int prime_reward;
    int kind;
} bgref_step_result;

int bgref_env_init(bgref_env* env, uint8_t* legal_boards, int max_legal_moves,
                   const int* dice, int n_dice);
int bgref_env_reset(bgref_env* env);
int bgref_env_step(bgref_env* env, int action, bgref_step_result* res);

/* ---- Philox4x32-10 + CPU self-play port (the bench's cpu_baseline) -------- */
void bgref_philox4x32(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo, uint32_t out[4]);

/* 1-ply self-play per the worker loop (src/multi/worker.py:78-174) on
 * n_threads host threads for about `seconds` wall seconds. Returns env steps
 * (pass steps included); *decisions, *episodes, *elapsed filled. */
long long bgref_selfplay_bench(const float* W1, const float* b1, const float* w2,
                               const float* b2, float temperature, uint64_t seed,
                               int n_threads, double seconds,
                               long long* decisions, long long* episodes,
                               double* elapsed);

/* The same loop with 2-ply scoring when ply == 2 (two_ply.py:44-150 exact
 * mode + the worker hook 153-193: the top 4 by V scored alpha*V - beta*W,
 * alpha 1.0, beta 0.9, softmax(score/T) over the four; 1-ply below 4 moves). */
long long bgref_selfplay_bench_ply(const float* W1, const float* b1, const float* w2,
                                   const float* b2, float temperature, uint64_t seed,
                                   int n_threads, double seconds, int ply,
                                   long long* decisions, long long* episodes,
                                   double* elapsed);
/* the same with `warmup` untimed env steps per thread first (whole games;
   BASELINE.md's CPU plan: a 300-step warm-up, then the timed window) */
long long bgref_selfplay_bench_warm(const float* W1, const float* b1, const float* w2,
                                    const float* b2, float temperature, uint64_t seed,
                                    int n_threads, double seconds, int ply, long long warmup,
                                    long long* decisions, long long* episodes,
                                    double* elapsed);

#ifdef __cplusplus
}
#endif
#endif
