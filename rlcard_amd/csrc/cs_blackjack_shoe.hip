// cs_blackjack_shoe.hip -- Blackjack with multi-deck shoes (2..8 decks) or 5..7 players: the tables the byte-ring
// kernel (cs_blackjack.h: one deck, at most 4 players) does not cover. Lane per env, like every other lane game.
//
// Reference: rlcard/games/blackjack/dealer.py:6-37 (deck = init_standard_deck() * num_decks unless num_decks is 0 or 1;
// np_random.shuffle(np.array(deck)); deal_card: idx = np_random.choice(len(deck)), deck.pop(idx) unless num_decks is 0),
// game.py:22-123 (two rounds of players 0..P-1 then the dealer; hit / stand; the dealer draws while < 17 after the last
// player), judger.py:2-73 (scores with soft aces, codes 2 / 1 / -1), envs/blackjack.py:38-103 (obs, payoffs).
//
// Why a separate path: a shoe of 5+ decks (260..416 cards) shuffles and deals with random_interval masks of 9 bits,
// which the byte ring (the low 8 bits of each tempered word, cs_ring.h) cannot serve. Here each env draws numpy's
// MT19937 words directly: the env's 624-word state is a column of the mt buffer (word k at mt[k * n + env], so the
// lanes of a wave reading the same position hit one line), twisted in-lane when consumed. The shoe is materialised
// (one byte per position, shuffled in place) and a removed-position mask makes deck.pop(idx) an order-statistic
// lookup. Not a BASELINE configuration: simple over fast (no MT staging, direct per-lane stores).
//
// Packed state, WORDS u32 words per env, word-major [WORDS][n]:
//   0        deck length (bits 0..8) | game pointer << 9 (3 bits) | over << 12
//   1        hand sizes of hands 0..5, 5 bits each (hand h = player h, hand P = the dealer)
//   2        hand sizes of hands 6..7 (bits 0..9) | winner codes 2 bits per player << 10 (0 none, 1 tie, 2 win, 3 loss)
//   3..15    removed positions of the shoe (416 bits)
//   16..119  the shuffled shoe: byte k = card id (init_standard_deck order: suit * 13 + rank, S H D C x A 2 .. K)
//   120..167 hands: hand h card k at byte 24 h + k
#include "cs_skeleton.h"

namespace cs {
namespace bjs {

constexpr int MAXP = 7, HAND_CAP = 24, MAXDECK = 52 * 8;
enum { W_META = 0, W_SZ0 = 1, W_SZ1 = 2, W_REMOVED = 3, W_DECK = 16, W_HANDS = 120, WORDS = 168 };
static_assert(W_DECK - W_REMOVED >= MAXDECK / 32 && W_HANDS - W_DECK >= MAXDECK / 4 &&
                  WORDS - W_HANDS >= (MAXP + 1) * HAND_CAP / 4, "state layout");

// word k of one env in a word-major array
struct Col {
    uint32_t* p;
    int64_t n;
    __device__ __forceinline__ uint32_t get(int k) const { return p[(int64_t)k * n]; }
    __device__ __forceinline__ void set(int k, uint32_t v) const { p[(int64_t)k * n] = v; }
    __device__ __forceinline__ uint32_t byte(int b) const { return (get(b >> 2) >> (8 * (b & 3))) & 255u; }
    __device__ __forceinline__ void set_byte(int b, uint32_t v) const
    {
        const uint32_t w = get(b >> 2), sh = 8u * (uint32_t)(b & 3);
        set(b >> 2, (w & ~(255u << sh)) | (v << sh));
    }
};

// numpy init_by_array (mt19937_init_by_array) into a column; the state then awaits its first twist
__device__ void init_by_array(const Col& mt, const uint32_t* key, int klen)
{
    uint32_t prev = 19650218u;
    mt.set(0, prev);
    for (int i = 1; i < MT_N; i++) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        mt.set(i, prev);
    }
    int i = 1, j = 0;
    prev = mt.get(0);
    for (int k = MT_N; k; k--) {
        const uint32_t v = (mt.get(i) ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        mt.set(i, v);
        prev = v;
        i++;
        j++;
        if (i >= MT_N) { mt.set(0, mt.get(MT_N - 1)); prev = mt.get(0); i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        const uint32_t v = (mt.get(i) ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        mt.set(i, v);
        prev = v;
        i++;
        if (i >= MT_N) { mt.set(0, mt.get(MT_N - 1)); prev = mt.get(0); i = 1; }
    }
    mt.set(0, 0x80000000u);
}

// the env's RandomState as plain words: pos = words of the current block consumed (MT_N: twist before the next)
struct WordRng {
    Col mt;
    uint32_t pos;
    __device__ void twist() const   // numpy's reload, in place (mt[k] reads mt[k + 1], mt[k + 397] / the new mt[k - 227])
    {
        for (int k = 0; k < MT_N - MT_M; k++) mt.set(k, mt_mix(mt.get(k), mt.get(k + 1), mt.get(k + MT_M)));
        for (int k = MT_N - MT_M; k < MT_N - 1; k++)
            mt.set(k, mt_mix(mt.get(k), mt.get(k + 1), mt.get(k + MT_M - MT_N)));
        mt.set(MT_N - 1, mt_mix(mt.get(MT_N - 1), mt.get(0), mt.get(MT_M - 1)));
    }
    __device__ __forceinline__ uint32_t next()
    {
        if (pos >= (uint32_t)MT_N) {
            twist();
            pos = 0;
        }
        return mt_temper(mt.get((int)pos++));
    }
    // random_interval(max): mask + rejection on whole tempered words (numpy legacy distributions.c)
    __device__ __forceinline__ uint32_t interval(uint32_t max)
    {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        do {
            v = next() & mask;
        } while (v > max);
        return v;
    }
};

__device__ __forceinline__ uint32_t card_tot(uint32_t c)   // judge value (A 11, J/Q/K 10) | ace << 8
{
    const uint32_t r = c % 13u;
    return r == 0 ? 11u + 256u : (r >= 9 ? 10u : r + 1u);
}
__device__ __forceinline__ int score_of(uint32_t t)        // judge_score from a total (cs_blackjack.h score_of)
{
    const int sc = (int)(t & 255u), aces = (int)(t >> 8);
    const int need = sc > 21 ? ((sc - 12) * 205) >> 11 : 0;
    return sc - 10 * (need < aces ? need : aces);
}

struct Shoe {
    Col s;
    int np, decks;

    __device__ __forceinline__ bool infinite() const { return decks == 0; }
    __device__ __forceinline__ int shoe_cards() const { return 52 * (decks >= 2 ? decks : 1); }
    __device__ __forceinline__ uint32_t meta() const { return s.get(W_META); }
    __device__ __forceinline__ int current() const { return (int)((meta() >> 9) & 7u); }
    __device__ __forceinline__ bool is_over() const { return (meta() >> 12) & 1u; }
    __device__ __forceinline__ int nhand(int h) const
    {
        return h < 6 ? (int)((s.get(W_SZ0) >> (5 * h)) & 31u) : (int)((s.get(W_SZ1) >> (5 * (h - 6))) & 31u);
    }
    __device__ __forceinline__ int winner(int p) const { return (int)((s.get(W_SZ1) >> (10 + 2 * p)) & 3u); }
    __device__ __forceinline__ int score(int h, int from) const
    {
        uint32_t t = 0;
        const int k1 = nhand(h);
        for (int k = from; k < k1; k++) t += card_tot(s.byte(4 * W_HANDS + HAND_CAP * h + k));
        return score_of(t);
    }
    __device__ __forceinline__ void add_card(int h, uint32_t c)
    {
        const int k = nhand(h);
        if (k >= HAND_CAP) return;   // a hand busts before 22 cards with <= 8 decks
        s.set_byte(4 * W_HANDS + HAND_CAP * h + k, c);
        if (h < 6) s.set(W_SZ0, s.get(W_SZ0) + (1u << (5 * h)));
        else s.set(W_SZ1, s.get(W_SZ1) + (1u << (5 * (h - 6))));
    }
    // deal_card: the idx-th remaining shoe position (idx = choice(len(deck))), removed unless the deck is infinite
    __device__ void deal(WordRng& rng, int h)
    {
        const uint32_t m = meta();
        const uint32_t len = m & 511u;
        uint32_t idx = rng.interval(len - 1u);
        const int total = shoe_cards();
        int pos = 0;
        for (int w = 0; w < (total + 31) / 32; w++) {
            const int valid = total - 32 * w;
            const uint32_t vm = valid >= 32 ? 0xFFFFFFFFu : ((1u << valid) - 1u);
            uint32_t fr = ~s.get(W_REMOVED + w) & vm;
            const uint32_t c = (uint32_t)__popc(fr);
            if (idx < c) {
                while (idx--) fr &= fr - 1u;
                pos = 32 * w + __builtin_ctz(fr);
                break;
            }
            idx -= c;
        }
        if (!infinite()) {
            s.set(W_REMOVED + (pos >> 5), s.get(W_REMOVED + (pos >> 5)) | 1u << (pos & 31));
            s.set(W_META, (m & ~511u) | (len - 1u));
        }
        add_card(h, s.byte(4 * W_DECK + pos));
    }
    __device__ void blank() const
    {
        s.set(W_META, 1u << 12);
        s.set(W_SZ0, 0u);
        s.set(W_SZ1, 0u);
    }
    // init_game (game.py:22-54): a fresh shoe, shuffled (Fisher-Yates i = len - 1 .. 1), then two rounds of
    // players 0..P-1 and the dealer
    __device__ void reset(WordRng& rng)
    {
        const int total = shoe_cards();
        for (int w = 0; w < total / 4; w++) {
            uint32_t v = 0;
            for (int b = 0; b < 4; b++) v |= (uint32_t)((4 * w + b) % 52) << (8 * b);
            s.set(W_DECK + w, v);
        }
        for (int i = total - 1; i >= 1; i--) {
            const int j = (int)rng.interval((uint32_t)i);
            if (j != i) {
                const uint32_t a = s.byte(4 * W_DECK + i), b = s.byte(4 * W_DECK + j);
                s.set_byte(4 * W_DECK + i, b);
                s.set_byte(4 * W_DECK + j, a);
            }
        }
        for (int w = 0; w < MAXDECK / 32; w++) s.set(W_REMOVED + w, 0u);
        s.set(W_SZ0, 0u);
        s.set(W_SZ1, 0u);
        s.set(W_META, (uint32_t)total);
        for (int r = 0; r < 2; r++) {
            for (int p = 0; p < np; p++) deal(rng, p);
            deal(rng, np);
        }
    }
    __device__ void finish(WordRng& rng)
    {
        while (score(np, 0) < 17) deal(rng, np);
        const int d = score(np, 0);
        uint32_t win = 0;
        for (int p = 0; p < np; p++) {
            const int sp = score(p, 0);
            const uint32_t code = sp > 21 ? 3u : (d > 21 ? 2u : (sp > d ? 2u : (sp < d ? 3u : 1u)));
            win |= code << (10 + 2 * p);
        }
        s.set(W_SZ1, (s.get(W_SZ1) & 0x3FFu) | win);
        s.set(W_META, (meta() & ~(7u << 9)) | 1u << 12);   // game pointer 0, over
    }
    __device__ void step(int a, WordRng& rng)                // game.py:56-123
    {
        const int gp = current();
        bool advance = true;
        if (a != 1) {   // anything but 'stand' hits
            deal(rng, gp);
            advance = score(gp, 0) > 21;
        }
        if (advance) {
            if (gp >= np - 1) finish(rng);
            else s.set(W_META, (meta() & ~(7u << 9)) | (uint32_t)(gp + 1) << 9);
        }
    }
    __device__ __forceinline__ uint32_t observe(int player) const   // [score(own), score(dealer visible)]
    {
        const int mine = score(player, 0);
        const int dealer = is_over() ? score(np, 0) : score(np, 1);
        return (uint32_t)mine | (uint32_t)dealer << 8;
    }
    __device__ __forceinline__ float payoff(int p) const
    {
        const int w = winner(p);
        return w == 2 ? 1.f : (w == 1 ? 0.f : -1.f);
    }
};

struct Lane {
    int64_t env;
    bool valid;
    Shoe g;
    WordRng rng;
};

__device__ __forceinline__ Lane lane_of(uint32_t* mt, uint32_t* st, const uint32_t* ctl, int64_t n, const GameParams& prm)
{
    Lane L;
    L.env = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    L.valid = L.env < n;
    const int64_t e = L.valid ? L.env : 0;
    L.g.s = Col{st + e, n};
    L.g.np = prm.num_players;
    L.g.decks = prm.num_decks;
    L.rng.mt = Col{mt + e, n};
    L.rng.pos = L.valid && ctl ? ctl[e] : 0u;
    return L;
}

__device__ __forceinline__ void emit(const Lane& L, const cs_step_out& out, int player, const float* r, int np,
                                     bool done)
{
    if (out.obs) ((uint16_t*)out.obs)[L.env] = (uint16_t)L.g.observe(player);
    if (out.legal) ((uint8_t*)out.legal)[L.env] = 3u;
    if (out.player) ((uint8_t*)out.player)[L.env] = (uint8_t)L.g.current();
    if (out.reward && r)
        for (int p = 0; p < np; p++) ((float*)out.reward)[L.env * np + p] = r[p];
    if (out.done) ((uint8_t*)out.done)[L.env] = (uint8_t)done;
}

// StepRecord (cs_engine.h): the env's state words, a system-scope fence, then the sequence number
__device__ __forceinline__ void record(const StepRecord& rec, const Lane& L)
{
    if (rec.seq == nullptr || !L.valid || L.env != rec.env) return;
    for (int w = 0; w < WORDS; w++) rec.words[w] = L.g.s.get(w);
    __threadfence_system();
    __hip_atomic_store(rec.seq, rec.seqv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(BLOCK) void k_seed(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                 const uint32_t* keys, const int32_t* klen, int64_t first,
                                                 int64_t count)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= count) return;
    const int64_t env = first + i;
    init_by_array(Col{mt + env, n}, keys + 2 * i, klen[i] == 2 ? 2 : 1);
    ctl[env] = (uint32_t)MT_N;   // numpy's state after seeding: the first draw twists
    Shoe g;
    g.s = Col{st + env, n};
    g.blank();
}

__global__ __launch_bounds__(BLOCK) void k_reset(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                  cs_step_out out, GameParams prm, StepRecord rec)
{
    Lane L = lane_of(mt, st, ctl, n, prm);
    if (!L.valid) return;
    L.g.reset(L.rng);
    const float r[MAXP] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    emit(L, out, L.g.current(), r, L.g.np, false);
    ctl[L.env] = L.rng.pos;
    record(rec, L);
}

__global__ __launch_bounds__(BLOCK) void k_step(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n,
                                                 const int32_t* actions, cs_step_out out, GameParams prm,
                                                 StepRecord rec)
{
    Lane L = lane_of(mt, st, ctl, n, prm);
    if (!L.valid) return;
    float r[MAXP] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool done = false;
    if (L.g.is_over()) {
        L.g.reset(L.rng);   // lazy auto-reset (include/cardsim.h cs_step)
    } else {
        L.g.step(actions[L.env], L.rng);
        done = L.g.is_over();
        if (done)
            for (int p = 0; p < L.g.np; p++) r[p] = L.g.payoff(p);
    }
    emit(L, out, L.g.current(), r, L.g.np, done);
    ctl[L.env] = L.rng.pos;
    record(rec, L);
}

__global__ __launch_bounds__(BLOCK) void k_observe(uint32_t* st, int64_t n, int player, cs_step_out out,
                                                    GameParams prm, StepRecord rec)
{
    Lane L = lane_of(nullptr, st, nullptr, n, prm);
    if (!L.valid) return;
    cs_step_out o = out;
    o.reward = nullptr;
    emit(L, o, player, nullptr, L.g.np, L.g.is_over());
    record(rec, L);
}

__global__ __launch_bounds__(BLOCK) void k_rollout(uint32_t* mt, uint32_t* ctl, uint32_t* st, int64_t n, int T,
                                                    uint64_t seed, uint64_t t0, uint64_t env_base, cs_traj_out out,
                                                    GameParams prm)
{
    Lane L = lane_of(mt, st, ctl, n, prm);
    if (!L.valid) return;
    const int np = L.g.np;
    if (L.g.is_over()) L.g.reset(L.rng);
    const uint64_t genv = env_base + (uint64_t)L.env;
    PolicyRng pol;
    for (int t = 0; t < T; t++) {
        const int64_t row = (int64_t)t * n + L.env;
        const int p = L.g.current();
        const uint32_t pr = pol.at(seed, genv, t0 + (uint64_t)t, t == 0);
        const int a = pick_legal32(3u, pr);
        ((uint16_t*)out.obs)[row] = (uint16_t)L.g.observe(p);
        ((uint8_t*)out.legal)[row] = 3u;
        ((uint8_t*)out.player)[row] = (uint8_t)p;
        ((uint8_t*)out.action)[row] = (uint8_t)a;
        L.g.step(a, L.rng);
        const bool done = L.g.is_over();
        float* rw = (float*)out.reward + row * np;
        for (int q = 0; q < np; q++) rw[q] = done ? L.g.payoff(q) : 0.f;
        ((uint8_t*)out.done)[row] = (uint8_t)done;
        if (done) {
            if (out.final_obs)   // Env.run's final state of every player (envs/env.py:161-164)
                for (int q = 0; q < np; q++) ((uint16_t*)out.final_obs)[row * np + q] = (uint16_t)L.g.observe(q);
            L.g.reset(L.rng);
        }
    }
    ctl[L.env] = L.rng.pos;
}

dim3 grid_of(int64_t n) { return dim3((unsigned)((n + BLOCK - 1) / BLOCK)); }

}  // namespace bjs

bool is_blackjack_shoe(const Buffers& b)
{
    return b.game == CS_GAME_BLACKJACK && (b.num_decks >= 2 || b.num_players > 4);
}

int bjs_game_info(const cs_config* cfg, cs_game_info* info)
{
    const int np = cfg && cfg->num_players > 0 ? cfg->num_players : 1;
    const int nd = cfg && cfg->num_decks >= 0 ? cfg->num_decks : 1;
    if (np > bjs::MAXP || nd > 8) return CS_E_UNSUPPORTED;
    if (cfg && cfg->rng_mode == CS_RNG_PHILOX) return CS_E_UNSUPPORTED;   // the Philox stream is bytes (cs_ring.h)
    info->obs_dim = 2;
    info->num_actions = 2;
    info->num_players = np;
    info->legal_bytes = 1;
    info->action_bytes = 1;
    info->state_words = bjs::WORDS;
    info->action_feature_dim = 2;
    info->rng_period = MT_N;   // position = words consumed of the current 624-word block
    info->game_words = bjs::WORDS;
    info->envs_per_wave = WAVE;   // k_rollout: one lane per env
    return CS_OK;
}

hipError_t bjs_launch_seed(const Buffers& b, const uint32_t* keys, const int32_t* klen, int64_t first, int64_t count,
                           hipStream_t s)
{
    hipLaunchKernelGGL(bjs::k_seed, bjs::grid_of(count), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, keys, klen,
                       first, count);
    return hipGetLastError();
}
hipError_t bjs_launch_reset(const Buffers& b, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(bjs::k_reset, bjs::grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, o, params_of(b),
                       b.rec);
    return hipGetLastError();
}
hipError_t bjs_launch_step(const Buffers& b, const int32_t* a, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(bjs::k_step, bjs::grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, a, o,
                       params_of(b), b.rec);
    return hipGetLastError();
}
hipError_t bjs_launch_observe(const Buffers& b, int32_t p, const cs_step_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(bjs::k_observe, bjs::grid_of(b.n), dim3(BLOCK), 0, s, b.state, b.n, p, o, params_of(b), b.rec);
    return hipGetLastError();
}
hipError_t bjs_launch_rollout(const Buffers& b, int32_t T, uint64_t seed, uint64_t t0, uint64_t env_base,
                              const cs_traj_out& o, hipStream_t s)
{
    hipLaunchKernelGGL(bjs::k_rollout, bjs::grid_of(b.n), dim3(BLOCK), 0, s, b.mt, b.ctl, b.state, b.n, T, seed, t0,
                       env_base, o, params_of(b));
    return hipGetLastError();
}

}  // namespace cs
