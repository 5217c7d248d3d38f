/* az_mcts.h — native lock-step MCTS engine (host C++, libaz_mcts.so).
 *
 * The caller side of the hot path: the search statistics and descent of the reference's
 * MCTS.search (MCTS.py:151-240) and the rules it calls per node (Connect4Game.py:116-219,
 * TicTacToeGame.py:60-200), for many concurrent games ("slots"), each with its own tree.
 * Leaf boards are handed out in batches for ONE network launch (predict_both on the
 * MI355X) and the results fed back, so the per-leaf host cost is native instead of Python
 * (SURVEY.md §8f ranks 1-2).
 *
 * Parity: every statistic keeps the reference's numeric type.  A Q value carries a tag
 * (Python int / Python float / np.float32) and is updated with NumPy 2 (NEP 50) promotion
 * rules, priors are float64 (float32 pi x int64 valids) normalised with NumPy's pairwise
 * summation, and UCB scores are float64 in the reference's operation order — so visit counts
 * and Q values equal the Python MCTS (itself pinned to the reference's traces) bit for bit
 * given the same network outputs (tests/test_native_mcts.py).
 *
 * Episode logic (temperature, move sampling with the game's RandomState, symmetries, the
 * expand_tree targets) stays in Python (mcts_native.py) and reads the root statistics back.
 *
 * Boards are int8 [n][n] in the reference's [x][y] order (board.tobytes() order), canonical
 * (player to move = +1).  Threading: az_mcts_collect may run the slots on `threads` host
 * threads; every other call is single-threaded per engine.  All calls return AZM_OK (0) or
 * a negative code with the text in az_mcts_last_error().
 */
#ifndef AZ_MCTS_H
#define AZ_MCTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZM_OK 0
#define AZM_EINVAL -1
#define AZM_ESTATE -2

#define AZM_GAME_CONNECT4 0   /* Connect4Game(board_size=n): n x n + pass, 4 in a row */
#define AZM_GAME_TICTACTOE 1  /* TicTacToeGame(n): n x n + pass, n in a row           */

/* Q value type tags (az_mcts_root_edges): the Python type the reference's Qsa holds. */
#define AZM_TAG_NONE -1       /* no (s, a) entry                                      */
#define AZM_TAG_INT 0         /* Python int                                           */
#define AZM_TAG_FLOAT 1       /* Python float (float64)                               */
#define AZM_TAG_F32 2         /* np.float32                                           */

typedef struct az_mcts az_mcts;

const char* az_mcts_last_error(void);

/* An engine for `slots` concurrent games of one kind.  n*n <= 64.  cpuct as args.cpuct;
 * use_gnn selects the GNN outputs for priors and leaf values (MCTS.py:172-193). */
az_mcts* az_mcts_create(int game, int n, int slots, double cpuct, int use_gnn);
void az_mcts_destroy(az_mcts* m);
int az_mcts_action_size(const az_mcts* m);

/* Fresh, empty tree for a slot (a new MCTS object, Coach.py:97). */
int az_mcts_reset(az_mcts* m, int slot);
/* getActionProb's reset of standard_predictions / gnn_predictions (MCTS.py:30-31). */
int az_mcts_clear_predictions(az_mcts* m, int slot);
/* Queue `sims` searches from the canonical root `board` (MCTS.py:33-34, 104-106). */
int az_mcts_begin(az_mcts* m, int slot, const int8_t* board, int sims);
/* Searches still to finish for a slot (a search waiting for its leaf counts). */
int az_mcts_remaining(const az_mcts* m, int slot);
/* The same for every slot at once: out[slots]. */
int az_mcts_remaining_all(const az_mcts* m, int32_t* out);
/* Drop a slot's queued searches (the tree keeps every finished simulation), so the caller
 * can recover after an exception it raised mid-search (AZ_STRICT_NN).  AZM_ESTATE while a
 * collected leaf is still waiting for its feed. */
int az_mcts_abandon(az_mcts* m, int slot);

/* Advance every slot with queued searches until it waits on a new leaf or has none left.
 * Writes up to `cap` leaf boards [n*n] and their slot ids, in ascending slot order; returns
 * the number written (>= 0) or an error code.  Terminal-only searches finish in here. */
int az_mcts_collect(az_mcts* m, int8_t* boards, int32_t* slots, int cap, int threads);

/* Network outputs for the leaves of the last collect, same order: pi/gpi [count][A] float32
 * probabilities, v/gv [count] float32 (gpi/gv may be NULL when use_gnn == 0).  failed != 0
 * applies the reference's exception path to every leaf (uniform priors, value 0,
 * MCTS.py:195-200).  Expands each leaf and backs its value up the searched path.
 * A failed request that was an episode slot's expand_tree root prediction is NOT degraded:
 * that predict is unguarded in the reference (MCTS.py:108-113), so the episode is aborted (it
 * is never reported finished).  Returns the number of episodes aborted this way (>= 0; the
 * caller raises the network's exception when it is non-zero) or an error code. */
int az_mcts_feed(az_mcts* m, int count, const float* pi, const float* v, const float* gpi,
                 const float* gv, int failed);

/* az_mcts_feed (network rows for the last collect, never failed) followed by az_mcts_collect, in
 * ONE parallel pass: each worker thread feeds a group of slots and runs their next descents back
 * to back.  Same trees and leaves as the two calls (every slot's work is independent of the
 * others').  Returns the new leaf count like az_mcts_collect.  A failed batch goes through
 * az_mcts_feed(failed = 1) instead.  cap must cover every slot that may hand out a leaf (fed,
 * searching or inside an episode; the slot count always does): a smaller cap fails with
 * AZM_EINVAL before any row is applied, so the same rows can still go through az_mcts_feed. */
int az_mcts_feed_collect(az_mcts* m, int count, const float* pi, const float* v,
                         const float* gpi, const float* gv, int8_t* boards, int32_t* slots,
                         int cap, int threads);

/* Speculative rows: network outputs of boards the search has not asked for yet (the arena
 * evaluates a leaf together with its children, mcts_native.ArenaPlayer), same layout as
 * az_mcts_feed.  A later search that reaches one of these boards as a new leaf is expanded from
 * the row inside az_mcts_collect instead of being handed out -- exactly what feeding that row
 * would do, so callers must only put rows bit-identical to the board's own evaluation.  The
 * cache is per engine, persists across az_mcts_reset / az_mcts_begin, and is read-only during a
 * collect.  az_mcts_cache_stats: out[0] = rows held, out[1] = leaves expanded from them. */
int az_mcts_cache_put(az_mcts* m, int count, const int8_t* boards, const float* pi, const float* v,
                      const float* gpi, const float* gv);
/* One slot's search step with speculation in one call pair (the arena, mcts_native.ArenaPlayer):
 * collect_spec advances `slot` to its next new leaf and writes it as boards[0], followed by up to
 * cap - 1 of its non-terminal children that are neither expanded in the tree nor cached; returns
 * the row count (0 when the slot's searches are done).  feed_spec takes the rows of those boards
 * in the same order: row 0 expands the leaf (as az_mcts_feed), rows 1.. go to the row cache.
 * failed != 0 applies the reference's exception path to the leaf and keeps no rows. */
int az_mcts_collect_spec(az_mcts* m, int slot, int8_t* boards, int cap);
int az_mcts_feed_spec(az_mcts* m, int count, const float* pi, const float* v, const float* gpi,
                      const float* gv, int failed);
int az_mcts_cache_clear(az_mcts* m);
int az_mcts_cache_stats(const az_mcts* m, int64_t* out);

/* Root statistics: nsa[A] visit counts (0 = no entry), q[A] values, qtag[A] AZM_TAG_*. */
int az_mcts_root_edges(const az_mcts* m, int slot, const int8_t* board, int32_t* nsa, double* q,
                       int8_t* qtag);
/* standard_predictions[s][1] when s is present in the current prediction epoch: returns 1 and
 * writes *v, else 0.  az_mcts_set_std records one (expand_tree's root predict, MCTS.py:108-113). */
int az_mcts_get_std(const az_mcts* m, int slot, const int8_t* board, float* v);
int az_mcts_set_std(az_mcts* m, int slot, const int8_t* board, float v);
/* Tree sizes of a slot: out[0] = len(Es), out[1] = len(Ns), out[2] = len(Ps), out[3] = sum(Nsa). */
int az_mcts_tree_stats(const az_mcts* m, int slot, int64_t* out);

/* Episode mode (Coach.executeEpisode, Coach.py:27-79, run natively per slot): a fresh tree and
 * np.random.RandomState(seed) for the slot; az_mcts_collect / az_mcts_feed then drive the
 * whole game (getActionProb with `sims` searches and its temp-0 tie-break, expand_tree with
 * `expand_by` searches when use_gnn, the move draw, the rules).  Requests from an episode slot
 * are leaves or, for expand_tree, the root's standard prediction (only v is used).  Finished
 * slots are reported once by az_mcts_episode_finished; az_mcts_episode_record copies the
 * per-move records (n = az_mcts_episode_moves): canonical boards [n][cells], player to move,
 * temp, action, pi [n][A] (float64; temp 0 one-hot), expand_tree root visits before/after
 * (nsa, has/tag, q) and the root's standard value, and getGameEnded's final value + type. */
int az_mcts_episode_begin(az_mcts* m, int slot, uint32_t seed, int sims, int expand_by,
                          int temp_threshold);
int az_mcts_episode_finished(az_mcts* m, int32_t* slots, int cap);
int az_mcts_episode_moves(const az_mcts* m, int slot);
int az_mcts_episode_record(const az_mcts* m, int slot, int8_t* boards, int8_t* curs,
                           int8_t* temps, int32_t* actions, double* pi, int32_t* init_nsa,
                           int8_t* init_has, float* std_v, int32_t* exp_nsa, double* exp_q,
                           int8_t* exp_tag, int* result_tag, double* result);
/* expand_tree's training targets of every recorded move of a finished episode (MCTS.py:115-146,
 * what Coach keeps as a GNN example): initial_policy and expanded_policy [n][A] (float64), and
 * expanded_value with its Python/NumPy type (AZM_TAG_INT / _FLOAT / _F32; the running sum and
 * the division follow the same NEP 50 promotions as the search's Q update).  A move whose root
 * had no visits before expansion gets valids / sum(valids). */
int az_mcts_episode_targets(const az_mcts* m, int slot, double* init_policy, double* exp_policy,
                            int8_t* exp_value_tag, double* exp_value);
/* Batched export for the self-play driver: moves[i] = az_mcts_episode_moves(slots[i]), and the
 * records (+ the targets when init_policy != NULL) of n finished slots written back to back into
 * arrays sized for sum(moves) (episode i starts at move sum(moves[:i])), result i at index i. */
int az_mcts_episodes_moves(const az_mcts* m, const int32_t* slots, int n, int32_t* moves);
int az_mcts_episode_records(const az_mcts* m, const int32_t* slots, int n, int8_t* boards,
                            int8_t* curs, int8_t* temps, int32_t* actions, double* pi,
                            int32_t* init_nsa, int8_t* init_has, float* std_v, int32_t* exp_nsa,
                            double* exp_q, int8_t* exp_tag, int* result_tags, double* results,
                            double* init_policy, double* exp_policy, int8_t* exp_value_tag,
                            double* exp_value);
/* np.random.RandomState emulation, for tests: op 0 = n raw uint32 draws, 1 = n x randint(0, np_),
 * 2 = n x choice(np_, p=p); az_rng_doubles = n x random_sample(). */
int az_rng_test(uint32_t seed, int op, int n, const double* p, int np_, int64_t* out);
int az_rng_doubles(uint32_t seed, int n, double* out);

/* Rules, exposed for differential tests against the Python games. ended: tag + value of
 * getGameEnded(board, 1); valids [A] int8; next: canonical board after action (player 1 moves,
 * then the board is seen from the opponent). */
int az_game_ended(int game, int n, const int8_t* board, int* tag, double* value);
int az_game_valids(int game, int n, const int8_t* board, int8_t* valids);
int az_game_next_canonical(int game, int n, const int8_t* board, int action, int8_t* out);
/* The non-terminal canonical boards one move below a non-terminal `board` (valid actions in
 * ascending order, at most `cap`), written to out [cap][n*n]; returns their count (0 for a
 * terminal board).  The arena's speculative leaf batches use it (mcts_native.ArenaPlayer). */
int az_game_children(int game, int n, const int8_t* board, int cap, int8_t* out);
/* np.sum of a float64 vector (NumPy's pairwise summation), for tests. */
double az_np_pairwise_sum(const double* a, int n);

#ifdef __cplusplus
}
#endif
#endif
