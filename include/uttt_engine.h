/*
 * uttt_engine.h — C ABI of the MI355X-native Ultimate Tic-Tac-Toe self-play engine.
 *
 * This is the drop-in boundary for the reference's native hot path
 * (cpp/uttt_game.h, cpp/uttt_mcts.h behind the pybind11 module `uttt_cpp`,
 * cpp/python_bindings.cpp:49-107). Plain C types only: pointers, sizes,
 * status codes. Every function returns UTTT_OK (0) or a negative UTTT_ERR_*;
 * uttt_last_error() gives the message of the calling thread's last failure.
 *
 * Two layers:
 *   1. Rules on one host-side state value (what `uttt_cpp.State` binds).
 *   2. The engine: thousands of PUCT trees in SoA arrays in HBM, advanced in
 *      lock-step rounds by HIP kernels (gfx950). A round = every unfinished
 *      tree descends to its next unevaluated leaf (absorbing terminal
 *      simulations), the leaves are handed to an evaluator as one NCHW batch,
 *      and the results are expanded + backed up. Self-play adds the per-move
 *      policy target, numpy-exact move sampling and game records on device.
 *
 * Semantics are those of cpp/uttt_mcts.cpp:84-196 bit for bit (see DESIGN.md,
 * "Exact semantics"); the only structural change is that the k identical
 * copies of a flushed leaf (uttt_mcts.cpp:121-135 queues the same leaf k times
 * because there is no virtual loss) are evaluated once and replayed k times.
 */
#ifndef UTTT_ENGINE_H
#define UTTT_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UTTT_OK 0
#define UTTT_ERR_ARG (-1)      /* invalid argument                                  */
#define UTTT_ERR_HIP (-2)      /* HIP runtime error                                 */
#define UTTT_ERR_CAPACITY (-3) /* node pool / path / record arena exhausted         */
#define UTTT_ERR_ORDER (-4)    /* call out of sequence (e.g. apply before select)   */
#define UTTT_ERR_NODEVICE (-5) /* no gfx950 device / device ordinal out of range    */
#define UTTT_ERR_NONFINITE (-6) /* evaluator returned NaN/Inf (legal prior or value) */

#define UTTT_ACTIONS 81
#define UTTT_MAX_SIMS 4095 /* most simulations per search (uttt_engine_create max_sims): the 16-byte node
                               record keeps N in 16 bits, k in 12, the first child in 20 */
#define UTTT_INPUT_SIZE 243 /* (3, 9, 9) NCHW f32 per position */

/* Packed, side-to-move-relative position (32 bytes; same bits on host and device).
 * own[w]/opp[w]: small boards 3w..3w+2, board b's 9 cells at bits 9*(b%3)..+8,
 *   so bit (a % 27) of word (a / 27) is action a = board*9 + cell.
 * mains: bits 0..8 main_board_pieces, bits 16..24 main_board_enemy_pieces.
 * active: -1 (any board) or 0..8.
 * Replaces UTTT::State's int arrays (cpp/uttt_game.h:49-54). */
typedef struct uttt_state {
    uint32_t own[3];
    uint32_t opp[3];
    uint32_t mains;
    int32_t active;
} uttt_state_t;

const char *uttt_last_error(void);
const char *uttt_version(void);

/* ---------------------------------------------------------------- rules --- */
/* State() — cpp/uttt_game.cpp:9-21 */
void uttt_state_initial(uttt_state_t *out);
/* State(pieces, enemy_pieces, main, main_enemy, active) — cpp/uttt_game.cpp:24-32.
 * Arrays are [board][cell] row-major. Values must be 0/1 and active in -1..8
 * (the reference does not validate; out-of-range input is UB there). */
int uttt_state_from_arrays(const int32_t pieces[81], const int32_t enemy_pieces[81],
                           const int32_t main_board_pieces[9], const int32_t main_board_enemy_pieces[9],
                           int32_t active_board, uttt_state_t *out);
/* get_pieces/... — cpp/uttt_game.h:42-46 */
void uttt_state_to_arrays(const uttt_state_t *s, int32_t pieces[81], int32_t enemy_pieces[81],
                          int32_t main_board_pieces[9], int32_t main_board_enemy_pieces[9],
                          int32_t *active_board);
/* State::next — cpp/uttt_game.cpp:97-145 (any action 0..80, unvalidated as in the reference) */
int uttt_state_next(const uttt_state_t *s, int32_t action, uttt_state_t *out);
/* State::legal_actions — cpp/uttt_game.cpp:148-191; returns the count, ascending actions in out */
int uttt_state_legal_actions(const uttt_state_t *s, int32_t out[81]);
/* is_lose / is_draw / is_done / is_first_player — cpp/uttt_game.cpp:77-94 (return 0/1) */
int uttt_state_is_lose(const uttt_state_t *s);
int uttt_state_is_draw(const uttt_state_t *s);
int uttt_state_is_done(const uttt_state_t *s);
int uttt_state_is_first_player(const uttt_state_t *s);
/* to_input_tensor — cpp/uttt_game.cpp:244-280 (HWC (9,9,3) flat) */
void uttt_state_input_hwc(const uttt_state_t *s, float out[243]);
/* The same for n states (out: n x 243 floats), e.g. the rank-0 .history build after a gather. */
int uttt_states_input_hwc(const uttt_state_t *s, int64_t n, float *out);
/* to_string — cpp/uttt_game.cpp:194-241; returns length, or -(needed) if cap too small */
int uttt_state_to_string(const uttt_state_t *s, char *buf, int32_t cap);
/* boltzman — cpp/uttt_mcts.cpp:199-216 */
int uttt_boltzman(const float *xs, int32_t n, float temperature, float *out);

/* --------------------------------------------------------------- engine --- */
typedef struct uttt_engine uttt_engine_t;

/* device: HIP ordinal (-1 = the calling thread's current device). max_trees: concurrent trees / game slots. max_sims: the
 * largest evaluate_count this engine will run, 1..4095 (sizes the node pool to the
 * exact worst case 82 + 81*max_sims nodes per tree, so it cannot overflow; the 16-byte node
 * record holds visits and child-block counts up to 4095). */
int uttt_engine_create(int32_t device, int32_t max_trees, int32_t max_sims, uttt_engine_t **out);
int uttt_engine_destroy(uttt_engine_t *eng);
/* Launch everything on `stream` (a hipStream_t, e.g. torch's current stream;
 * NULL = the null stream). Until called, the engine uses a stream of its own. */
int uttt_engine_set_stream(uttt_engine_t *eng, void *stream);
/* The engine's own non-blocking stream (created with the engine; each engine's
 * stream gets its own hardware queue when few streams exist), e.g. to run an
 * evaluator on it so that several engines on one GPU overlap. */
int uttt_engine_own_stream(uttt_engine_t *eng, void **stream);
/* Device bytes held by the engine. */
int64_t uttt_engine_device_bytes(const uttt_engine_t *eng);

/* Search semantics for uttt_search_begin_mode:
 *  UTTT_SEMANTICS_CPP  cpp/uttt_mcts.cpp (pv_mcts_cpp / self_play_cpp): root
 *                      pre-expanded uniform, expand appends k blocks, f32 PUCT;
 *  UTTT_SEMANTICS_PY   pv_mcts.py (evaluate_network / evaluate_best_player):
 *                      root evaluated by the first flush, expand replaces,
 *                      PUCT as NumPy 2 evaluates the Python expression
 *                      (float32 with sqrt in double; float64 where the
 *                      all-zero-prior fallback made the priors float64). */
#define UTTT_SEMANTICS_CPP 0
#define UTTT_SEMANTICS_PY 1
/* Start a search of n_trees independent trees (pv_mcts_scores,
 * uttt_mcts.cpp:92-103: root expanded with uniform priors 1/|legal|).
 * roots: host array of n_trees states. */
int uttt_search_begin(uttt_engine_t *eng, const uttt_state_t *roots, int32_t n_trees, int32_t evaluate_count,
                      int32_t batch_size);
/* The same with explicit semantics (replaces pv_mcts.py:133-181 when PY). */
int uttt_search_begin_mode(uttt_engine_t *eng, const uttt_state_t *roots, int32_t n_trees, int32_t evaluate_count,
                           int32_t batch_size, int32_t semantics);

/* One round of descents (uttt_mcts.cpp:109-127). Writes the pending leaves'
 * network inputs, NCHW (n,3,9,9) f32, to device memory nn_input (room for
 * max_trees*243 floats; may be NULL) in deterministic tree order, and stores
 * the number of pending leaves in *n_pending (0 = search finished). Blocks on
 * the stream to read the count. */
int uttt_search_select(uttt_engine_t *eng, float *nn_input, int32_t *n_pending);

/* The same round without reading the count on the host: launches the descents and the
 * pending-leaf scan and returns at once. The count stays on the device (uttt_search_count_ptr:
 * [0] pending leaves, [1] trees stopped by the select budget); uttt_nn_stem, the *_dev network
 * entry points and uttt_search_apply (device results, one row per leaf) read it there, so a
 * round is enqueued with no host synchronisation. A round whose count is 0 changes nothing:
 * the caller enqueues rounds until a count it copied back (uttt_search_count_copy) reads
 * [2] == 0: no tree has simulations left once this round is applied (the next select would
 * report 0). Replaces the per-round blocking read of uttt_search_select for the self-play
 * driver. */
int uttt_search_select_async(uttt_engine_t *eng);
/* Enqueue a copy of the round's counts to dst[0..2] (host, pinned for an asynchronous copy):
 * [0] pending leaves, [1] trees stopped by the select budget, [2] trees with simulations left
 * after this round's apply. */
int uttt_search_count_copy(uttt_engine_t *eng, int32_t *dst);
/* Device address of the round's counts. */
int uttt_search_count_ptr(uttt_engine_t *eng, const int32_t **count);
/* uttt_search_select_async whose scan also stores the three counts into slot ring_slot (0..7) of
 * the engine's host-visible count ring (fine-grained pinned memory, system-scope stores): the host
 * reads them once an event recorded after this call has completed, with no copy on the stream. */
int uttt_search_select_async_to(uttt_engine_t *eng, int32_t ring_slot);
/* The same, and the scan stores `tag` into word 3 of the slot after the counts (a system-scope release
 * store): the host polls the tag instead of an event (round 5, SelfPlay's network rounds). */
int uttt_search_select_async_tag(uttt_engine_t *eng, int32_t ring_slot, int32_t tag);
/* The count ring: *ring = n_slots x {pending, stopped, left after apply, tag} int32, host memory. */
int uttt_search_count_ring(uttt_engine_t *eng, const int32_t **ring, int32_t *n_slots);

/* Host copies of the pending leaves (slot order) and their multiplicity k
 * (the number of identical copies the reference would have queued). */
int uttt_search_pending(uttt_engine_t *eng, uttt_state_t *states, int32_t *copies);
/* One-tree searches (the drop-in uttt_cpp.pv_mcts_scores, python_bindings.cpp:83-100 / uttt_mcts.cpp:109-167)
 * without a copy operation or a stream synchronisation per flush (round 5): select_host launches the
 * select and the scan, which stores the counts, the pending leaf's state and its copies k into fine-grained
 * pinned host memory and then a tag the host spins on; apply_host copies the leaf's evaluation (81 priors
 * by action, value; one row or one per copy) into pinned host memory that k_apply reads directly, and
 * returns without waiting. Same results as uttt_search_select + uttt_search_pending + uttt_search_apply. */
int uttt_search_select_host(uttt_engine_t *eng, uttt_state_t *leaf, int32_t *copies, int32_t *n_pending);
int uttt_search_apply_host(uttt_engine_t *eng, const float *policy, int64_t policy_stride, const float *value,
                           int32_t rows);  /* rows: 1 (one result for the leaf's k copies) or k (one per copy,
                                              applied in order: the reference's call pattern) */

/* A one-tree search as ONE resident wave (round 6; replaces the reference's pv_mcts_scores loop,
 * uttt_mcts.cpp:84-196, as python_bindings.cpp:11-47 drives it, for uttt_cpp.pv_mcts_scores): search1_begin
 * launches the wave (root expansion included), which descends to the first flush's leaf and hands it over
 * through fine-grained pinned memory; search1_next waits for it (n_pending 1: *leaf and its copies k) or for
 * the search's end (n_pending 0; the tree's error status is raised here); search1_apply writes the leaf's
 * evaluation (one row for the k copies, or k rows in order) and a command the wave polls, and returns
 * without waiting; search1_scores copies the root's scores (pv_mcts_scores' return value: one-hot at
 * temperature 0, else boltzman, as uttt_search_scores) the wave stored at the end. No launch, copy or
 * stream synchronisation per flush; a wave left without a command for 100 ms exits and search1_next
 * resumes it. Same results as uttt_search_begin + uttt_search_select_host / apply_host + scores. */
int uttt_search1_begin(uttt_engine_t *eng, const uttt_state_t *root, int32_t sims, int32_t batch, int32_t semantics,
                       float temperature);
int uttt_search1_next(uttt_engine_t *eng, uttt_state_t *leaf, int32_t *copies, int32_t *n_pending);
int uttt_search1_apply(uttt_engine_t *eng, const float *policy, int64_t policy_stride, const float *value,
                       int32_t rows);
int uttt_search1_scores(uttt_engine_t *eng, float *scores, int32_t *n_legal);
/* Diagnostics (no reference counterpart): the resident wave's own time split up to its last hand-over, in
 * 10 ns ticks since its launch: [0] descents, [1] applies, [2] waits for the host's commands. */
int uttt_search1_time_split(uttt_engine_t *eng, int32_t *ticks3);

/* Evaluator results for the pending leaves (uttt_mcts.cpp:138-167: legal-mask,
 * sequential f32 renormalisation, expand k times, back up k times).
 * Row r of policy (>= 81 f32, stride policy_ld) / value (stride value_ld)
 * belongs to pending slot r. per_copy != 0: the rows are per queued copy
 * (slot 0's k copies first, then slot 1's ...), as the reference's model()
 * batch is. on_device: pointers are device (else host, copied on the stream). */
int uttt_search_apply(uttt_engine_t *eng, const float *policy, int64_t policy_ld, const float *value,
                      int64_t value_ld, int32_t per_copy, int32_t on_device);

/* Deterministic hash evaluator on device (test / micro-benchmark evaluator;
 * DESIGN.md "Hash evaluator"): n rows of nn_input -> policy (n,81), value (n). */
int uttt_eval_hash(uttt_engine_t *eng, const float *nn_input, int32_t n, float *policy, float *value);
/* The same evaluator on the round's pending leaves read from their states, the count read on the
 * device (after uttt_search_select_async): rows [0, count) of policy (81 f32 each) and value. */
int uttt_eval_hash_dev(uttt_engine_t *eng, float *policy, float *value);
/* One whole round with the hash evaluator, enqueued by one call (round 5; the rounds of
 * SelfPlay.steps with HashEvaluator lanes, i.e. the kernel microbenchmark of SURVEY §8(d)):
 * uttt_search_select_async_to(ring_slot) -> uttt_eval_hash_dev(policy, value) ->
 * uttt_search_apply(on_device), with the apply staged: the next call runs it and its own select as
 * one launch (k_round: per tree, the previous evaluation applied, then the next descent), and any
 * other call that reads the trees (the move's end, the root results, a synchronous select) applies
 * it first. UTTT_FUSED_ROUNDS=0 launches the three steps as written above. The scan stores the
 * round's counts and then `tag` (word 3 of the slot; the counts' stores drained before it), so the host
 * learns that the counts landed by polling the tag: no event and no host sync per round. policy:
 * (max_trees, 81) f32, value: (max_trees,) f32, device memory, left untouched until the staged apply
 * has run. Replaces, for the test evaluator, one pass of the flush loop of uttt_mcts.cpp:109-167
 * over every tree. */
int uttt_round_hash_async(uttt_engine_t *eng, int32_t ring_slot, int32_t tag, float *policy, float *value);
/* n_rounds consecutive rounds in one call (round 6, tree-only self-play: the host's per-round reaction was
 * the bound): ring slots ring_slot .. ring_slot + n_rounds - 1 (mod 8) and tags tag .. tag + n_rounds - 1;
 * a round past the move's last finds every tree done and changes nothing. */
int uttt_rounds_hash_async(uttt_engine_t *eng, int32_t ring_slot, int32_t tag, float *policy, float *value,
                           int32_t n_rounds);
/* A move's whole round loop in one call (round 6; replaces, for the test evaluator, the flush loop of
 * uttt_mcts.cpp:109-167 run to the move's end over every tree, as self_play_cpp.play's per-move
 * pv_mcts_scores call does): `depth` hash rounds kept in flight (uttt_round_hash_async, ring slots from
 * ring_slot on, tags tag, tag + 1, ... masked to 31 bits), the host spinning on each round's tag in turn and
 * enqueueing the next until a round reports no tree with simulations left. Returns when that round's
 * counts landed; the rounds still in flight behind it are empty. *n_rounds: rounds enqueued (ring slots and
 * tags consumed), *n_leaves: leaves evaluated, *n_with_leaves: rounds that had leaves. */
int uttt_rounds_hash_move(uttt_engine_t *eng, int32_t ring_slot, int32_t tag, float *policy, float *value,
                          int32_t depth, int32_t *n_rounds, int64_t *n_leaves, int32_t *n_with_leaves);

/* Root results after the search: visit counts of the root's children (legal
 * order, row stride 81) and |legal| per tree. */
int uttt_search_root_visits(uttt_engine_t *eng, int32_t *visits, int32_t *n_legal);
/* Scores as pv_mcts_scores returns them (uttt_mcts.cpp:177-195): one-hot first
 * max for temperature 0, else boltzman; row stride 81. */
int uttt_search_scores(uttt_engine_t *eng, float temperature, float *scores, int32_t *n_legal);

/* -------------------------------------------------------------- self-play --- */
/* Self-play of games [game_begin, game_end) (self_play_cpp.py:34-130), each
 * game g with its own numpy-legacy MT19937 seeded seed_base + g (=
 * np.random.seed(seed_base + g) before self_play_cpp.play). Slots are refilled
 * with the next game id as games end. arena_plies bounds the finished-game
 * record arena (plies). */
int uttt_selfplay_begin(uttt_engine_t *eng, int64_t game_begin, int64_t game_end, uint32_t seed_base,
                        float temperature, int32_t evaluate_count, int32_t batch_size, int64_t arena_plies);
/* Start one move for every live game: its search tree is rebuilt from the
 * current position (no tree reuse, uttt_mcts.cpp:92). *n_live = live slots
 * (0 = every game finished). Then run select/eval/apply rounds. */
int uttt_selfplay_move_begin(uttt_engine_t *eng, int32_t *n_live);
/* Finish the move (self_play_cpp.py:63-92): scores -> f64 policy target
 * (np.sum renormalisation) -> np.random.choice -> record -> next state;
 * ended games get their values (self_play_cpp.py:95-99) and are written to
 * the arena; free slots take the next game. *n_finished = games in the arena. */
int uttt_selfplay_move_end(uttt_engine_t *eng, int64_t *n_finished);
/* numpy-legacy MT19937 state of a slot's current game (624 words + position),
 * so a caller can run a game on numpy's global RandomState and continue it
 * afterwards (self_play_cpp.play draws from np.random, self_play_cpp.py:86). */
int uttt_selfplay_get_rng(uttt_engine_t *eng, int32_t slot, uint32_t key[624], int32_t *pos);
int uttt_selfplay_set_rng(uttt_engine_t *eng, int32_t slot, const uint32_t key[624], int32_t pos);
/* The move boundary without host synchronisation, for a driver that pipelines moves
 * (DESIGN.md §7): uttt_selfplay_move_end_async enqueues the move's end (scores, sampled move,
 * records, new games for free slots) and a copy of the counters to pinned host memory;
 * uttt_selfplay_move_begin_async enqueues the next move's roots (the live flags stay on the
 * device). Once the stream has passed that copy (e.g. an event recorded after it completed),
 * uttt_selfplay_move_result reports failed trees and a full arena, as move_end does, and
 * returns the games finished so far and the live slots of the next move. Not with periodic
 * cache clears (uttt_engine_set_cache clear_every > 0). */
int uttt_selfplay_move_begin_async(uttt_engine_t *eng);
int uttt_selfplay_move_end_async(uttt_engine_t *eng);
int uttt_selfplay_move_result(uttt_engine_t *eng, int64_t *n_finished, int32_t *n_live_next);

/* Finished games: n_games entries of (game id, first ply in arena, plies),
 * sorted by game id; then the arena rows [0, n_plies): state, policy target
 * (81 f64), action, value. Any output pointer may be NULL. */
int uttt_selfplay_games(uttt_engine_t *eng, int64_t *game_ids, int64_t *offsets, int32_t *lengths,
                        int64_t max_games, int64_t *n_games);
int uttt_selfplay_plies(uttt_engine_t *eng, uttt_state_t *states, double *policies, int8_t *actions,
                        int8_t *values, float *inputs_hwc, int64_t max_plies, int64_t *n_plies);

/* ----------------------------------------------------- evaluation cache --- */
/* Use `owner`'s evaluation table instead of a private one (several engines on
 * one GPU, e.g. SelfPlay lanes, then see each other's evaluations). Lookups and
 * inserts are coherent across concurrently running kernels; only the owner
 * clears the table (its clear_every_moves). The owner must outlive `eng`. */
int uttt_engine_share_cache(uttt_engine_t *eng, uttt_engine_t *owner);
/* Position -> raw evaluator output table in HBM (2^log2_capacity entries of
 * 360 B; 0 = off, the default). A flushed leaf whose position is cached is
 * expanded from the table inside the select kernel instead of waiting for the
 * evaluator. Exact for a deterministic evaluator (the evaluator sees only the
 * position, uttt_game.cpp:244-280). Self-play clears it at begin and every
 * clear_every_moves moves (0 = never); per-copy apply bypasses it. */
int uttt_engine_set_cache(uttt_engine_t *eng, int32_t log2_capacity, int32_t clear_every_moves);
int uttt_engine_cache_clear(uttt_engine_t *eng);
/* hits: leaves resolved from the table; misses: leaves sent to the evaluator. */
int uttt_engine_cache_stats(uttt_engine_t *eng, int64_t *hits, int64_t *misses, int64_t *inserts);
/* The same plus replacements: inserts that found every probe slot holding another position and
 * rewrote one of them (a full probe window; readers of the old entry retry). */
int uttt_engine_cache_stats2(uttt_engine_t *eng, int64_t *hits, int64_t *misses, int64_t *inserts,
                             int64_t *replacements);

/* ------------------------------------------------------------ telemetry --- */
/* Per-kernel timing with HIP events on the engine's stream (off by default). */
int uttt_engine_set_timing(uttt_engine_t *eng, int32_t enabled);
/* kernel: 0 select, 1 apply, 2 encode, 3 scan, 4 move_end, 5 hash_eval.
 * Outputs total ms, launches and algorithmic bytes. Counters without launches
 * (value in *algo_bytes): 6 tree levels walked by select (sum over descents of depth + 1),
 * 7 trees that descended, 9 sum over select launches of the slowest tree's levels. */
int uttt_engine_kernel_stats(uttt_engine_t *eng, int32_t kernel, double *total_ms, int64_t *launches,
                             int64_t *algo_bytes);
int uttt_engine_reset_stats(uttt_engine_t *eng);

#ifdef __cplusplus
}
#endif

#endif /* UTTT_ENGINE_H */
