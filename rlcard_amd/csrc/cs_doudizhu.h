// cs_doudizhu.h -- DouDizhu: constants, action-table layout and packed env state shared by the host table builder
// (cs_ddz_table.cpp) and the kernels (cs_doudizhu.hip).
//
// Reference: rlcard/games/doudizhu/{dealer,round,game,judger,player,utils}.py and rlcard/envs/doudizhu.py
// (SURVEY.md 8(a) A15-A17). Unlike the 2-4 action games, DouDizhu runs ONE WAVE PER ENV: a step scans the
// 27 472-id action table against the hand and writes 901 + 3 434 bytes, work for 64 lanes, while the game logic
// itself is a handful of wave-uniform (scalar) updates.
//
// Cards are only ranks (suits never matter in DouDizhu): rank r = 0..14 for 3,4,...,K,A,2,black joker,red joker.
// A multiset of cards = 15 nibbles (count 0..4 at bits 4r..4r+3) in a u64 ("packed counts"), so
//   contains(hand, combo)   = (((hand | H) - combo) & H) == H     with H = bit 3 of every nibble  (no borrow escapes)
//   hand -= combo / played += combo are plain 64-bit subtract / add.
#pragma once
#include <stdint.h>

namespace cs {
namespace ddz {

constexpr int NA = 27472;         // action ids (envs/doudizhu.py:20-21): 27 471 card combos + pass
constexpr int PASS = 27471;
constexpr int ND = (NA + 31) / 32;  // 859 mask dwords
constexpr int OBS = 901;          // peasant obs; the landlord's 790 are zero-padded to 901 (envs/doudizhu.py:40-47)
constexpr int OBS_LANDLORD = 790;
constexpr int LB = (NA + 7) / 8;  // 3 434 legal bytes per row
constexpr int P = 3;
constexpr int WORDS = 36;         // packed state words per env (env-major 144-B rows, see below)
constexpr int MAX_GROUPS = 320;   // (type, weight) groups: 308 in the reference table, scanned 64 per wave pass
constexpr int TYPE_BOMB = 35, TYPE_ROCKET = 36;  // indices in tools/gen_ddz_table.py TYPE_NAMES
constexpr uint32_t NONE = 3;      // "no player" for greater_player / winner
constexpr uint32_t NO_ACTION = 0xFFFFu;
constexpr uint64_t NIB_HI = 0x0888888888888888ull;  // bit 3 of the 15 rank nibbles

// Device action table, built once per handle from the table compiled into the library (ddz_actions.bin):
//   cnt[id]     packed counts of the combo (pass: 0)
//   gid[id]     its (type, weight) group
//   grp[g]      {gmin lo, gmin hi, start | end << 16, type_end | type << 16 | weight << 24}: the group's id range
//               [start, end), the end of its type's id range, and gmin = the elementwise minimum of the group's counts
//               (a hand that does not contain gmin contains no combo of the group: the legal-set scan skips it)
//   drange[d]   first | last << 16: the groups holding ids [32d, 32d + 32) (ids < PASS only)
// Every type is one contiguous id range with non-decreasing weights (checked by the builder), so "same type, greater
// weight" (utils.py:590-621 get_gt_cards) is the id range [grp[gid[prev]].end, type_end).
struct Tab {
    const uint64_t* cnt;
    const uint16_t* gid;
    const uint32_t* grp;     // [MAX_GROUPS][4]
    const uint32_t* drange;  // [ND]
    int32_t ng;
    int32_t bomb_lo, bomb_hi, rocket;
    int32_t bomb_g;          // group of the first bomb (bombs and the rocket: groups bomb_g .. bomb_g + 13)
    // kfirst[k]: the first id of group 32 k (PASS past the last group): the ids of groups 32 k .. 32 k + 31 lie in
    // [kfirst[k], kfirst[k + 1]), so a 32-group pass of the legal scan that no candidate range meets is skipped
    int32_t kfirst[MAX_GROUPS / 32 + 1];
};

// "Simple" ids, whose packed counts and group the kernels compute instead of loading them from the table (checked by
// the table builder): solo / pair / trio of rank r = ids r / 15 + r / 28 + r (groups = ids), bomb of rank r = bomb_lo
// + r, the rocket (groups bomb_g + r, bomb_g + 13).
constexpr uint32_t SIMPLE_HI = 41;
#ifdef __HIPCC__
#define CS_DDZ_HD __host__ __device__ __forceinline__
#else
#define CS_DDZ_HD inline
#endif
CS_DDZ_HD bool simple_id(uint32_t id, uint32_t bomb_lo)
{
    return id < SIMPLE_HI || id - bomb_lo <= 13u;
}
CS_DDZ_HD uint64_t simple_cnt(uint32_t id, uint32_t bomb_lo)
{
    const uint32_t k = id < 15u ? 1u : (id < 28u ? 2u : (id < SIMPLE_HI ? 3u : 4u));
    const uint32_t r = id < 15u ? id : (id < 28u ? id - 15u : (id < SIMPLE_HI ? id - 28u : id - bomb_lo));
    return r == 13u && id >= SIMPLE_HI ? (1ull << 52 | 1ull << 56) : (uint64_t)k << (4u * r);
}
CS_DDZ_HD uint32_t simple_gid(uint32_t id, uint32_t bomb_lo, uint32_t bomb_g)
{
    return id < SIMPLE_HI ? id : bomb_g + (id - bomb_lo);
}

// Packed env state (u32 words, env-major: st[env * WORDS + w]):
//   0..5   hand[p]   packed counts, p = 0 (landlord), 1, 2     (lo, hi)
//   6..11  played[p] packed counts                              (Round.played_cards, round.py:67-79)
//   12..16 the last 9 trace action ids, u16 each, oldest first; NO_ACTION = not yet played ('' padding,
//          envs/doudizhu.py:107-119). Trace entry i was played by player i % 3 (landlord opens, next = (p + 1) % 3).
//   17     number of trace entries (game.py:65 round.trace)
//   18     greater_player | greater_player's last play id << 16   (player.py:60-108, round.py:54-65)
//   19     current player | winner << 8                            (game.py:66-81; winner NONE = not over)
//   20..33 the dealt deck: byte k = the card at shuffled position k (sorted-deck id: rank * 4 + suit S H D C for
//          rank < 13, 52 black joker, 53 red joker; dealer.py:12-76). Written at the deal, read by the host only:
//          the suit-level hands and seen_cards of raw_obs / get_perfect_information (player.py:46-58, round.py:25-39)
//   34, 35 zero (16-B rows)
enum { W_HAND = 0, W_PLAYED = 6, W_HIST = 12, W_NTRACE = 17, W_GREATER = 18, W_CUR = 19, W_DECK = 20 };
constexpr int DECK_BYTES = 4 * (WORDS - W_DECK);   // 64: bytes 54..63 zero

// The state k_seed writes (lane per env, like every other game): a finished game (winner 0), so the next
// reset/step deals.
struct SeedView {
    static constexpr int SCRATCH_WORDS = 0;
    static constexpr bool RING = false;   // doudizhu keeps the two-block word layout (cs_doudizhu.hip)
    template <class Prm>
    __host__ __device__ void bind(uint32_t*, const Prm&) {}
    __host__ __device__ void blank() {}
    __host__ __device__ void store(uint32_t* st, int64_t, int64_t env) const
    {
        uint32_t* w = st + env * WORDS;
        for (int k = 0; k < WORDS; k++) w[k] = 0;
        for (int k = W_HIST; k < W_HIST + 5; k++) w[k] = 0xFFFFFFFFu;
        w[W_GREATER] = NONE;
        w[W_CUR] = 0u | (0u << 8);
    }
};

#ifdef __HIPCC__
// _cards2array (envs/doudizhu.py:150-166) of packed counts: bit 4r + k = (count_r > k) for r < 13, bit 52 / 53 = jokers
__device__ __forceinline__ uint64_t cards_bits(uint64_t c)
{
    const uint64_t lo = c & 0x000FFFFFFFFFFFFFull, H = 0x0008888888888888ull;
    const uint64_t t = (((lo + 0x0007777777777777ull) & H) >> 3) | (((lo + 0x0006666666666666ull) & H) >> 2) |
                       (((lo + 0x0005555555555555ull) & H) >> 1) | ((lo + 0x0004444444444444ull) & H);
    return t | ((uint64_t)(((c >> 52) & 15u) != 0) << 52) | ((uint64_t)(((c >> 56) & 15u) != 0) << 53);
}
#endif

}  // namespace ddz
}  // namespace cs
