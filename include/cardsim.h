/*
 * cardsim.h -- C ABI of the MI355X-native batched card-game engine (rlcard_amd).
 *
 * The reference (pmcgannon22/rlcard) has no FFI: its env path is pure Python. This ABI is the
 * boundary a binding (ctypes here: rlcard_amd/_abi.py; cgo/JNI/N-API stubs in INTEGRATION.md) calls to replace,
 * for a whole batch of envs at once, the reference calls listed per entry point. POD types only, 64-bit sizes,
 * no exceptions across the boundary: every call returns CS_OK (0) or a negative CS_E_* code, and
 * cs_last_error() returns a thread-local message for the last failure on the calling thread.
 *
 * Ownership: env state and the per-env MT19937 streams live in device memory owned by the handle. Every output
 * buffer is caller-owned DEVICE memory (e.g. torch tensors' data_ptr()) with the documented shape/dtype, C-contiguous.
 * All work is enqueued asynchronously on the caller's hipStream_t (`stream`, NULL = default stream); a handle is not
 * thread-safe: drive it from one stream/thread. One handle per GPU.
 */
#ifndef RLCARD_AMD_CARDSIM_H
#define RLCARD_AMD_CARDSIM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    CS_OK = 0,
    CS_E_INVALID = -1,   /* bad argument (null pointer, size, config) */
    CS_E_DEVICE = -2,    /* HIP runtime error (no device, launch failure, out of memory) */
    CS_E_STATE = -3,     /* call out of order (e.g. reset before seed) */
    CS_E_UNSUPPORTED = -4
};

/* game ids; names as registered by rlcard/envs/__init__.py:6-54 */
enum { CS_GAME_BLACKJACK = 0, CS_GAME_LEDUC = 1, CS_GAME_LIMIT = 2, CS_GAME_DOUDIZHU = 3, CS_GAME_NOLIMIT = 4 };

typedef struct cs_handle cs_handle;

/* Game configuration: the 'game_*' keys Env.__init__ forwards to Game.configure (rlcard/envs/env.py:33-39). */
typedef struct {
    int32_t num_players; /* blackjack 'game_num_players' (default 1); leduc/limit/no-limit 2; doudizhu 3 (0 = default) */
    int32_t num_decks;   /* blackjack 'game_num_decks' (default 1, 0 = infinite); ignored elsewhere (-1 = default) */
    int32_t chips_for_each; /* no-limit 'chips_for_each' (nolimitholdem/game.py:45-56): stack, 1..255 (0 = 100) */
    int32_t dealer_plus1;   /* no-limit 'dealer_id' + 1: 0 = None (drawn by the first game, then kept), 1..N fixed */
    int32_t rng_mode;       /* CS_RNG_MT19937 (0): every env draws numpy's RandomState stream of its seed, bit-exact
                               with the reference; CS_RNG_PHILOX (1): a counter-based Philox4x32-10 byte stream keyed
                               by the same seed key -- same games and rules, NOT the reference's deals; no MT19937
                               state traffic (every game; doudizhu draws the same byte stream) */
    int32_t reserved[3];
} cs_config;

enum { CS_RNG_MT19937 = 0, CS_RNG_PHILOX = 1 };

/* Static shape of a game (rlcard Env.num_players / num_actions / state_shape). */
typedef struct {
    int32_t obs_dim;      /* bytes per obs row: leduc 36, limit 72, no-limit 54, blackjack 2, doudizhu 901 (landlord 790) */
    int32_t num_actions;  /* leduc/limit 4, no-limit 5, blackjack 2, doudizhu 27472 */
    int32_t num_players;
    int32_t legal_bytes;  /* ceil(num_actions / 8): legal-action bitmask bytes per row */
    int32_t action_bytes; /* dtype width of rollout action rows: 1 (uint8) or 2 (int16, doudizhu) */
    int32_t state_words;  /* packed u32 words of game state per env */
    int32_t action_feature_dim; /* bytes per cs_action_features row: doudizhu 54, otherwise num_actions (one-hot) */
    int32_t rng_period;   /* draws after which the stream position of cs_get_rng_ctl wraps: doudizhu 1 248 (two word
                             blocks), the others the byte ring's 9 984 (16 slots of 624) */
    int32_t game_words;   /* packed game words at the start of the state_words (cs_get_env_state); = state_words for
                             every game without a deal queue */
    int32_t deal_queue_depth; /* DQ: deals the rollout may draw ahead (heads-up Limit / No-limit hold'em: 8 in this
                             build; 0 = no queue). state_words = game_words + 1 + 2 * DQ when DQ > 0; layout at
                             cs_get_env_state */
    int32_t envs_per_wave; /* envs one 64-lane wave of cs_rollout plays (doudizhu 2, heads-up Limit / No-limit 32,
                             otherwise 64): the write pattern cs_traj_probe reproduces */
} cs_game_info;
/* cs_game_info grows at its end between ABI versions (2: game_words, deal_queue_depth, envs_per_wave; 3 adds the
 * cs_state_* functions); a consumer built against this header checks cs_abi_version() >= CS_ABI_VERSION before
 * calling cs_game_info_get, which writes sizeof(cs_game_info) bytes of this version. */
#define CS_ABI_VERSION 3

/* Outputs of reset/step/observe, all device pointers, one row per env:
 *   obs    uint8  [n][obs_dim]     the current player's observation (values 0/1; blackjack: the two scores;
 *                                  no-limit: 52 card bits, then my chips and the largest chips in the pot)
 *   legal  uint8  [n][legal_bytes] legal-action bitmask, bit a of byte a/8 (LSB first) = action id a
 *   player uint8  [n]              current player id (Env.get_player_id)
 *   reward float  [n][num_players] payoffs of the transition (non-zero only where done; Env.get_payoffs). f32 of the
 *                                  reference's float64 payoffs, and exact for every payoff a game can reach: Leduc
 *                                  (judger.py:50-56) splits total / #winners among at most 2 winners (2 cards per
 *                                  rank; 3..5 players included), so its payoffs are multiples of 0.25; hold'em pays
 *                                  whole chips (/ 2 big blinds in Limit), Blackjack +-1 / 0, DouDizhu 0 / 1
 *                                  (tests/test_reward_precision.py enumerates them)
 *   done   uint8  [n]              1 if the game is over after this call (Env.is_over)
 * Any pointer may be NULL to skip that output. */
typedef struct {
    void* obs;
    void* legal;
    void* player;
    void* reward;
    void* done;
} cs_step_out;

/* Rollout trajectory, all device pointers, rows [T][n]:
 *   obs [T][n][obs_dim] u8, legal [T][n][legal_bytes] u8, player [T][n] u8 (the acting player's pre-step view),
 *   action [T][n] (uint8 or int16 per cs_game_info.action_bytes), reward [T][n][num_players] f32, done [T][n] u8,
 *   final_obs [T][n][num_players][obs_dim] u8 OPTIONAL (NULL = skip): where done[t][e] = 1, every player's observation
 *   of the finished game (the final states Env.run appends, envs/env.py:161-164); other rows are not written. */
typedef struct {
    void* obs;
    void* legal;
    void* player;
    void* action;
    void* reward;
    void* done;
    void* final_obs;
} cs_traj_out;

/* Transitions of a rollout trajectory, all device pointers [T][n] (any may be NULL to skip it):
 *   next_t i32   row of the acting player's next observation in the same game (obs[next_t][e]); -1 = the game ended
 *                first (next state = final_obs[end_t][e][player]); -2 = the game continues past the window
 *   end_t  i32   row where the row's game ends, -1 = past the window
 *   reward f32   the acting player's payoff on its last transition of the game, else 0
 *   done   u8    1 on that last transition
 *   ret    f32   the acting player's payoff of the game (DMC target), NaN if the game ends past the window */
typedef struct {
    void* next_t;
    void* end_t;
    void* reward;
    void* done;
    void* ret;
} cs_trans_out;

/* Shape of a game under a config. Replaces reading Env.num_players / num_actions / state_shape. */
int cs_game_info_get(int32_t game, const cs_config* cfg, cs_game_info* info);

/* Create n envs of `game` on HIP device `device`. Replaces rlcard.make(env_id, config) (envs/registration.py:77-89)
 * for n independent envs; allocates state (state_words*4 B/env) + the MT19937 streams in HBM: lane games' byte ring
 * 12 480 B/env (624 block words + 16 x 624 ring bytes), doudizhu 4 992 B/env, Blackjack shoes 2 496 B/env. */
int cs_create(cs_handle** out, int32_t game, int64_t num_envs, int32_t device, const cs_config* cfg);
void cs_destroy(cs_handle* h);

/* Seed envs [first_env, first_env + n) from init_by_array keys computed on the host from each env's seed
 * (rlcard/utils/seeding.py:33-113): keys [n][2] u32 (HOST memory), key_len [n] (1 or 2). Replaces Env.seed(seed)
 * (envs/env.py:228-231). Marks those envs as finished (the next reset/step starts a game). */
int cs_seed(cs_handle* h, const uint32_t* keys, const int32_t* key_len, int64_t first_env, int64_t n, void* stream);

/* Start a new game in every env. Replaces Env.reset() (envs/env.py:52-63) -> Game.init_game + _extract_state. */
int cs_reset(cs_handle* h, const cs_step_out* out, void* stream);

/* One Env.step (envs/env.py:65-86) per env with actions [n] int32 (DEVICE memory). Illegal ids follow the
 * reference's _decode_action (envs/leducholdem.py:81-96, limitholdem.py:81-96). Envs whose game was already over
 * start a new game instead (lazy auto-reset: action ignored, done = 0, reward = 0), so an RL loop never calls
 * reset() per env. */
int cs_step(cs_handle* h, const int32_t* actions, const cs_step_out* out, void* stream);

/* Observation of `player` in every env without changing state. Replaces Env.get_state(player_id)
 * (envs/env.py:188-197), e.g. the final states Env.run appends for every player (env.py:161-164). */
int cs_observe(cs_handle* h, int32_t player, const cs_step_out* out, void* stream);

/* T fused lockstep steps with an in-kernel uniform-random policy over the legal actions (the random-agent
 * benchmark policy of examples/run_random.py, agents/random_agent.py:17-47, with the global np.random replaced by
 * Philox4x32-10 keyed by (policy_seed) on counter (env_base + env, t0 + t)). A finished game restarts immediately.
 * Replaces T iterations of the Env.run loop (envs/env.py:120-169) for every env. */
int cs_rollout(cs_handle* h, int32_t T, uint64_t policy_seed, uint64_t t0, uint64_t env_base, const cs_traj_out* out,
               void* stream);

/* Placement probe of a trajectory allocation: zeros written into every non-NULL tensor of `out` ([T][n] rows, the
 * cs_rollout layout) in the rollout's write order, without game logic or state change. Where a trajectory lands in HBM
 * sets how fast it takes the rollout's writes (the same kernel runs 14 % slower in some allocations, and
 * this probe's time separates them exactly), so a caller can time it on a few candidate allocations and keep the
 * fastest (rlcard_amd.VecEnv.new_traj_out(select=k)). No reference counterpart (an allocation policy of this engine). */
int cs_traj_probe(cs_handle* h, int32_t T, const cs_traj_out* out, void* stream);

/* The whole engine state of a handle's envs -- MT streams, control words, game state, the rollout's staged stream rows
 * -- as one device buffer of cs_state_bytes bytes: cs_state_save copies it out, cs_state_load back in (async on
 * `stream`, device-to-device). A save / rollout / load sequence leaves the envs exactly as they were: how
 * rlcard_amd.VecEnv.new_traj_out times a real rollout on each candidate trajectory allocation without moving the
 * envs. The analogue of the reference's whole-game snapshot for step_back (rlcard/envs/env.py:88-106, the game's
 * deepcopy history), for every env at once. Since ABI version 3. */
int cs_state_bytes(const cs_handle* h, int64_t* bytes);
int cs_state_save(cs_handle* h, void* buf, void* stream);
int cs_state_load(cs_handle* h, const void* buf, void* stream);

/* rlcard's reorganize (utils/utils.py:153-179: per player [state, action, reward, next_state, done]) and the DMC
 * return target (agents/dmc_agent/utils.py:97-163) of a cs_rollout trajectory of this handle, on the device. `traj`
 * needs player, reward and done. Games still running at the end of the window come out as next_t = -2. */
int cs_transitions(cs_handle* h, int32_t T, const cs_traj_out* traj, const cs_trans_out* out, void* stream);

/* Legal-action id lists of `rows` legal bitmask rows of this game (wavefront compaction; the keys of
 * state['legal_actions']): counts i32 [rows], offsets i64 [rows + 1] (exclusive prefix sum, offsets[rows] = total),
 * ids i32 [total] ascending per row. ids may be NULL: size it from offsets[rows], then call again with it. */
int cs_legal_lists(cs_handle* h, const void* legal, int64_t rows, int32_t* counts, int64_t* offsets, int32_t* ids,
                   void* stream);

/* Action features of `count` action ids (Env.get_action_feature: doudizhu _cards2array of the combo, 54 B,
 * envs/doudizhu.py:136-142; other games one-hot of num_actions, envs/env.py:211-220): u8 [count][action_feature_dim]. */
int cs_action_features(cs_handle* h, const int32_t* ids, int64_t count, void* features, void* stream);

/* Chance-sampling CFR on Leduc Hold'em (rlcard/agents/cfr_agent.py:30-123) over this handle's envs: `iterations` x
 * CFRAgent.train(). Per iteration, for each player, every env deals a new game from its own stream (Env.reset) and
 * the whole betting tree under that deal is traversed with the reference's step / step_back recursion (traverse_tree),
 * accumulating regrets and the average policy; then regret matching updates the policy (update_policy). Tables are
 * caller-owned DEVICE buffers indexed by the Leduc observation the reference keys its dicts with
 * (((hand * 4 + public + 1) * 15 + my chips) * 15 + others' chips, 2700 rows): policy / average_policy / regrets
 * double [2700][4] (policy initialised to 0.25 = the reference's row for an unseen key), flags uint32 [2700] (bit 0:
 * key in policy, bit 1: key in regrets and average_policy), zero-initialised. iteration0 = the agent's iteration
 * count before this call. A 1-env handle is the reference agent, bit-exact (same fp64 operation order); with more
 * envs, each deals its own game per player per iteration and the tables add the deals' terms in one fixed order
 * (records sorted by infoset, then a sequential sum per segment: bit-exact with the oracle and run to run,
 * cs_cfr.hip). Leduc only. */
int cs_cfr_train(cs_handle* h, int32_t iterations, int64_t iteration0, double* policy, double* average_policy,
                 double* regrets, uint32_t* flags, void* stream);

/* ---- DMC learner side (rlcard/agents/dmc_agent/) ----------------------------------------------------------------
 * Actor buffers (utils.py:97-163 act): every (env, player) of a handle keeps its stream of transitions -- state = the
 * obs the player acted on (int8 [obs_dim]), action = Env.get_action_feature of its action (int8 [action_feature_dim]),
 * target = the player's payoff of that game on each of its rows, done / episode_return set on its last row of the
 * game -- and a T-row chunk is handed out once more than T rows of finished games are queued (`while size[p] > T`).
 * The streams live in a ring of `slots` chunks per (env, player) in HBM. Chunk ids handed out by cs_dmc_fill must be
 * gathered (cs_dmc_gather) before the next cs_dmc_fill reuses their slots; rows that would overwrite a chunk still
 * held are dropped and flagged (cs_dmc_status). Needs slots * T >= T + the rows one fill adds per (env, player) +
 * the longest game's rows. */
typedef struct cs_dmc cs_dmc;

/* get_batch (utils.py:33-46) output, DEVICE pointers, [T][B] rows (any may be NULL):
 *   state int8 [T][B][state_dim(player)] (doudizhu landlord 790, peasants 901), action int8 [T][B][feature_dim],
 *   target float [T][B], done uint8 [T][B], episode_return float [T][B] */
typedef struct {
    void* state;
    void* action;
    void* target;
    void* done;
    void* episode_return;
} cs_dmc_batch;

int cs_dmc_create(cs_handle* h, int32_t T, int32_t slots, cs_dmc** out);
void cs_dmc_destroy(cs_dmc* d);
/* Append the rows of a trajectory of this handle (cs_rollout layout [T_roll][n]; needs obs, player, action, reward,
 * done; player >= num_players marks a row that is not a transition) to the streams, in time order. The chunks that
 * become ready are listed in ready (int64 [cap], DEVICE) as ids, in (env, player, chunk) order; *nready (int64,
 * DEVICE) = their number (entries past cap are not written). Replaces the per-actor act loop for every env at once. */
int cs_dmc_fill(cs_dmc* d, int32_t T_roll, const cs_traj_out* traj, int64_t* ready, int64_t cap, int64_t* nready,
                void* stream);
/* get_batch: `count` chunk ids (DEVICE int64, all of player `player`) stacked along dim 1 into `out`. */
int cs_dmc_gather(cs_dmc* d, int32_t player, const int64_t* chunks, int64_t count, const cs_dmc_batch* out,
                  void* stream);
/* Synchronous, sticky flags: bit 0 = rows were dropped because a stream's ring was full (slots too few, or chunks not
 * gathered) -- those streams are broken (no chunk holding a dropped row is ever listed, later rows of the stream are
 * dropped too); bit 1 = a fill had more ready chunks than `cap` (the rest are listed by the next fill). */
int cs_dmc_status(cs_dmc* d, uint32_t* host_flags);

/* DMCNet scoring of legal actions (model.py:21-43 forward, 91-110 predict), first layer fused: for entry i (state
 * state_of[i], action ids[i]) h1[i] = relu(X[state_of[i]] + b1 + W_act . feature(ids[i])), X = W_obs . obs precomputed
 * per state ([S][H] float), W_act float [feature_dim][H] (the first Linear's action columns, transposed), b1 [H],
 * h1 float [E][H]; H a multiple of 4. Features as cs_action_features. All DEVICE memory. */
int cs_dmc_layer1(cs_handle* h, const float* X, const int32_t* state_of, const int32_t* ids, int64_t E, int32_t H,
                  const float* W_act, const float* b1, float* h1, void* stream);
/* Per state s (legal entries [offsets[s], offsets[s] + counts[s]) of values / ids, cs_legal_lists layout): the id with
 * the largest value (np.argmax: first maximum), or with probability eps a uniform legal id (DMCAgent.step; Philox
 * keyed by seed on (state_base + s, t) in place of np.random). actions int32 [S], -1 where a state has no entry. */
int cs_dmc_select(const float* values, const int32_t* counts, const int64_t* offsets, const int32_t* ids, int64_t S,
                  float eps, uint64_t seed, uint64_t t, uint64_t state_base, int32_t* actions, void* stream);

/* Copy the packed state words of env `env` (state_words u32, HOST buffer) -- the raw fields behind
 * Env.get_state()['raw_obs'] / get_perfect_information for single-env compatibility and debugging. Synchronous.
 * Heads-up Limit and No-limit hold'em (cs_game_info.deal_queue_depth = DQ > 0): words [0, game_words) are the game,
 * then the env's deal queue -- deals the rollout drew ahead from the env's stream, oldest first, that the next games
 * will use -- as one header word H and DQ entries of two words (entry k at words game_words + 1 + 2k, +2 + 2k). With
 * CB = log2(DQ) + 1 and XB = 2 CB - 1 (DQ 8: CB 4, XB 7; DQ 4: CB 3, XB 5):
 *   H bits [0, CB)        number of queued deals (0..DQ)
 *   H bits [CB, 2CB - 1)  slot of the oldest queued deal; queued deal i (i < count) is in slot (head + i) % DQ
 *   H bit XB, XB + 1      No-limit only: the dealer seat has been drawn / the drawn dealer seat
 *   H bits XB + 2 + 2k, XB + 3 + 2k   bits 8..7 of slot k's draw count
 *   e0 (first word of a slot) bits 25..31  bits 6..0 of the slot's draw count: MT19937 words the deal consumed
 *                                          (saturating at 511), so the env's position in its own game stream is the
 *                                          cs_get_rng_ctl position minus the queued deals' draw counts
 * Other bits of the entries are the engine's packed deal (holes, board, blind seat) -- opaque to a consumer. */
int cs_get_env_state(cs_handle* h, int64_t env, uint32_t* host_words, int32_t nwords);

/* Asynchronous cs_get_env_state: the state words of env `env` copied on `stream` into dst (u32 [state_words],
 * DEVICE memory), so a single-env host can bring them back with its step outputs in one transfer (rlcard_amd.make's
 * Env: one packed device-to-host copy per Env.step, envs/env.py:65-86). */
int cs_copy_env_state(cs_handle* h, int64_t env, uint32_t* dst, void* stream);

/* Single-env completion without a stream synchronisation (rlcard_amd.make's Env: one launch and a spin per Env.step):
 * when seq is not NULL, every later cs_reset / cs_step / cs_observe also writes env `env`'s packed state words to
 * `words` (state_words u32, 16-byte aligned) and then -- after a system-scope fence ordering all of that env's output
 * stores -- the call's sequence number to *seq: 1 for the first call after cs_set_step_record, then 2, 3, ... Both
 * are device-visible pointers, typically mapped pinned host memory the host polls. seq NULL turns it off. Only that
 * env's outputs are covered; meant for single-env handles. */
int cs_set_step_record(cs_handle* h, int64_t env, uint32_t* words, uint32_t* seq);

/* Overwrite the packed state words of env `env` from a HOST buffer taken by cs_get_env_state: Env.step_back
 * (envs/env.py:88-108) restores the game from its history. The env's RNG stream is left where it is, as the
 * reference's history does not hold np_random for most games (Blackjack's does: cs_load_env_rng). Synchronous. */
int cs_set_env_state(cs_handle* h, int64_t env, const uint32_t* host_words, int32_t nwords);

/* An env's whole RNG stream (numpy RandomState: position word + MT19937 block words / byte ring) as *words u32, for
 * the state a deep copy of the reference's RandomState holds. cs_copy_env_rng copies env `env`'s stream into dst,
 * cs_load_env_rng writes it back from src (both DEVICE memory, asynchronous on `stream`). Blackjack's Game.step
 * deep-copies the dealer -- its np_random included -- before every step and Game.step_back restores that copy
 * (rlcard/games/blackjack/game.py:66-70, 125-135), so the reference's redraws after a step back replay the undone
 * cards: rlcard_amd.make's Blackjack Env snapshots the stream with its history and loads it on step_back. */
int cs_env_rng_words(cs_handle* h, int32_t* words);
int cs_copy_env_rng(cs_handle* h, int64_t env, uint32_t* dst, void* stream);
int cs_load_env_rng(cs_handle* h, int64_t env, const uint32_t* src, void* stream);

/* Stream position (u32 draws consumed) bookkeeping word of env `env` (HOST out). Synchronous; for parity tests.
 * The position is ctl & 0x3FFF (DouDizhu: ctl & 0x7FF), the draws consumed modulo cs_game_info.rng_period; the other
 * bits are the engine's. Hold'em envs with a deal queue: the position includes the draws of the queued deals (their
 * counts are decoded as cs_get_env_state documents; tools/abi_driver.c). */
int cs_get_rng_ctl(cs_handle* h, int64_t env, uint32_t* host_ctl);

/* Evaluator test hook: the value the hold'em kernels' showdown evaluator gives `n` 7-card hands (Hand.evaluateHand +
 * the tie-break of compare_hands, limitholdem/utils.py:3-614): cards int8 [n][7] card2index ids (suit * 13 + rank,
 * S H D C x A 2 .. K; DEVICE), values uint32 [n] (DEVICE): category << 20 | five 4-bit tie-break ranks -- larger
 * wins, equal splits. No handle: the evaluator is stateless. */
int cs_debug_holdem_rank7(const int8_t* cards, int64_t n, uint32_t* values, void* stream);

/* DouDizhu legal-set test hook: the legal-action bitmask the step / rollout kernels build, for `n` (hand, previous
 * play) cases: counts u8 [n][15] (cards per rank 3 .. A, 2, black joker, red joker), prev i32 [n] (the largest play
 * on the table, made by another player; < 0 = leading) -> legal u8 [n][3434] (bit = id, pass included when
 * following). All DEVICE memory. Replaces Judger.playable_cards_from_hand (doudizhu/judger.py:124-258) /
 * get_gt_cards (doudizhu/utils.py:225-262). Needs a doudizhu handle (its action table). */
int cs_debug_ddz_legal(cs_handle* h, const uint8_t* counts, const int32_t* prev, int64_t n, uint8_t* legal,
                       void* stream);

/* Testing hook: when enabled, the wave-cooperative MT refill is skipped, so every block crossing takes the in-lane
 * serial twist; results must be identical. */
int cs_debug_set_serial_refill(cs_handle* h, int32_t enable);

/* Tuning hook: kernel variant bits (bit 0 = serial MT refill; DouDizhu rollouts: every legal set through the group
 * pass, no following fast path; bit 1 = DouDizhu rollouts: the whole legal image zeroed at every step; bit 2 = dword
 * instead of 16-B obs stores). Results are identical for every value. */
int cs_debug_set_kernel_flags(cs_handle* h, int32_t flags);

const char* cs_last_error(void);
const char* cs_version(void);
int32_t cs_abi_version(void);   /* CS_ABI_VERSION of the library */

#ifdef __cplusplus
}
#endif
#endif
