// san_driver.cpp -- AddressSanitizer + UndefinedBehaviorSanitizer run over the host-side C/C++: the CPU
// oracle (oracle/*.c, every game through create / seed / reset / step / observe / rollout, CFR, the evaluator and the
// DouDizhu legal-set KAT hook), the C ABI's host code (include/cardsim.h entry points on their argument-validation and
// no-device paths; cs_abi.cpp) and the DouDizhu table expansion (cs_ddz_table.cpp table_build_host). Built by
// `make -C tools san_driver` with -fsanitize=address,undefined on those sources only (the HIP kernels are linked
// unsanitized: GPU sanitizers are not available here). Test infrastructure; run by tests/test_sanitizers.py.
// Exit 0 = every check passed and no sanitizer report (reports abort: -fno-sanitize-recover).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "../include/cardsim.h"
#include "../oracle/oracle.h"
#include "../rlcard_amd/csrc/cs_doudizhu.h"

namespace cs {
namespace ddz {
std::string table_build_host(std::vector<uint8_t>& host, size_t off[4], Tab* tab);
}
}  // namespace cs

extern "C" void or_ddz_set_table(const uint8_t* counts, const int16_t* type, const int16_t* weight, int bomb,
                                 int rocket);
extern "C" void or_ddz_legal_kat(const uint8_t* hand15, int greater_play, uint8_t* bits);

static int fails = 0;
#define EXPECT(c)                                                            \
    do {                                                                     \
        if (!(c)) {                                                          \
            fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);   \
            fails++;                                                         \
        }                                                                    \
    } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 11);
}

// the oracle's DouDizhu table, from the library's compiled one (the pytest path loads it from the reference's npz)
static void oracle_ddz_table(const std::vector<uint8_t>& host, const size_t off[4])
{
    const uint64_t* cnt = (const uint64_t*)(host.data() + off[0]);
    std::vector<uint8_t> counts((size_t)cs::ddz::NA * 15);
    for (int id = 0; id < cs::ddz::NA; id++)
        for (int r = 0; r < 15; r++) counts[(size_t)id * 15 + r] = (uint8_t)((cnt[id] >> (4 * r)) & 15);
    std::vector<int16_t> type(cs::ddz::NA, -1), weight(cs::ddz::NA, -1);
    const uint32_t* grp = (const uint32_t*)(host.data() + off[2]);
    const uint16_t* gid = (const uint16_t*)(host.data() + off[1]);
    for (int id = 0; id < cs::ddz::PASS; id++) {
        const uint32_t w = grp[(size_t)gid[id] * 4 + 3];
        type[id] = (int16_t)((w >> 16) & 0xFF);
        weight[id] = (int16_t)(w >> 24);
    }
    or_ddz_set_table(counts.data(), type.data(), weight.data(), cs::ddz::TYPE_BOMB, cs::ddz::TYPE_ROCKET);
}

// the oracle: every game, every entry point, outputs sized exactly as oracle.h documents them
static void oracle_games()
{
    const int games[] = {OR_BLACKJACK, OR_LEDUC, OR_LIMIT, OR_DOUDIZHU, OR_NOLIMIT};
    for (int g : games) {
        for (int variant = 0; variant < 2; variant++) {
            or_cfg cfg = {0, 1, 100, -1, 0};
            cfg.num_players = g == OR_BLACKJACK ? (variant ? 3 : 1) : (g == OR_DOUDIZHU ? 3 : 2);
            if (g == OR_BLACKJACK && variant) cfg.num_decks = 0;
            if (g == OR_NOLIMIT && variant) { cfg.chips_for_each = 7; cfg.dealer_id = 1; }
            or_info info;
            EXPECT(or_game_info(g, &cfg, &info) == 0);
            const int64_t n = g == OR_DOUDIZHU ? 6 : 40;
            const int T = g == OR_DOUDIZHU ? 40 : 300;
            or_batch* b = or_batch_create(g, n, &cfg);
            EXPECT(b != nullptr);
            std::vector<uint32_t> keys(n * 2);
            std::vector<int32_t> klen(n);
            for (int64_t i = 0; i < n; i++) {
                keys[2 * i] = rnd();
                keys[2 * i + 1] = rnd();
                klen[i] = 1 + (int)(i & 1);
            }
            or_batch_seed(b, keys.data(), klen.data());
            const int O = info.obs_dim, LB = info.legal_bytes, P = info.num_players;
            std::vector<uint8_t> obs(n * O), legal(n * LB), player(n), done(n);
            std::vector<float> reward(n * P);
            or_batch_reset(b, obs.data(), legal.data(), player.data(), reward.data(), done.data());
            std::vector<int32_t> act(n);
            for (int s = 0; s < 60; s++) {
                for (int64_t i = 0; i < n; i++) act[i] = (int32_t)(rnd() % (uint32_t)(info.num_actions + 2)) - 1;
                or_batch_step(b, act.data(), obs.data(), legal.data(), player.data(), reward.data(), done.data());
                for (int p = 0; p < P; p++) or_batch_observe(b, s % n, p, obs.data(), legal.data());
            }
            std::vector<uint8_t> tobs((size_t)T * n * O), tleg((size_t)T * n * LB), tpl((size_t)T * n),
                tdone((size_t)T * n), fin((size_t)T * n * P * O);
            std::vector<int32_t> tact((size_t)T * n);
            std::vector<float> trew((size_t)T * n * P);
            or_batch_rollout(b, T, 5, 0, 0, tobs.data(), tleg.data(), tpl.data(), tact.data(), trew.data(),
                             tdone.data(), fin.data());
            or_batch_rollout(b, T, 5, T, 0, tobs.data(), tleg.data(), tpl.data(), tact.data(), trew.data(),
                             tdone.data(), nullptr);
            EXPECT(or_batch_draws(b, 0) > 0);
            or_batch_destroy(b);
        }
    }
}

static void oracle_cfr_and_kats()
{
    uint32_t keys[4] = {42, 0, 7, 0};
    int32_t klen[2] = {1, 1};
    or_cfr* c = or_cfr_create(2, keys, klen);
    or_cfr_train(c, 3);
    std::vector<double> pol(OR_CFR_INFOSETS * 4), avg(OR_CFR_INFOSETS * 4), reg(OR_CFR_INFOSETS * 4);
    std::vector<uint8_t> flags(OR_CFR_INFOSETS);
    or_cfr_tables(c, pol.data(), avg.data(), reg.data(), flags.data());
    EXPECT(or_cfr_draws(c, 0) > 0);
    or_cfr_destroy(c);

    for (int k = 0; k < 2000; k++) {   // 7 distinct cards
        int8_t cards[7];
        uint64_t used = 0;
        for (int j = 0; j < 7; j++) {
            int x;
            do x = (int)(rnd() % 52); while ((used >> x) & 1);
            used |= 1ull << x;
            cards[j] = (int8_t)x;
        }
        EXPECT((or_holdem_rank7(cards) >> 20) >= 1 && (or_holdem_rank7(cards) >> 20) <= 9);
    }

    std::vector<uint8_t> bits(cs::ddz::LB);
    for (int k = 0; k < 300; k++) {
        uint8_t hand[15] = {0};
        const int ncards = 1 + (int)(rnd() % 20);
        for (int j = 0; j < ncards; j++) {
            const int r = (int)(rnd() % 15);
            if (hand[r] < (r >= 13 ? 1 : 4)) hand[r]++;
        }
        memset(bits.data(), 0, bits.size());
        or_ddz_legal_kat(hand, (k & 1) ? (int)(rnd() % cs::ddz::PASS) : -1, bits.data());
    }
}

// the ABI's host paths that run without a GPU: shapes, argument validation, error strings, no-device failure
static void abi_host()
{
    cs_game_info info;
    cs_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.num_decks = -1;
    for (int g = 0; g < 5; g++) EXPECT(cs_game_info_get(g, &cfg, &info) == CS_OK && info.obs_dim > 0);
    EXPECT(cs_game_info_get(7, &cfg, &info) != CS_OK);
    EXPECT(cs_game_info_get(CS_GAME_LEDUC, &cfg, nullptr) == CS_E_INVALID);
    // Blackjack shoes / big tables (cs_blackjack_shoe.hip): 8 decks x 7 players; 9 decks, 8 players and the
    // Philox byte stream are refused
    cfg.num_players = 7;
    cfg.num_decks = 8;
    EXPECT(cs_game_info_get(CS_GAME_BLACKJACK, &cfg, &info) == CS_OK && info.state_words == 168 && info.num_players == 7);
    cfg.num_decks = 9;
    EXPECT(cs_game_info_get(CS_GAME_BLACKJACK, &cfg, &info) == CS_E_UNSUPPORTED);
    cfg.num_decks = 2;
    cfg.num_players = 8;
    EXPECT(cs_game_info_get(CS_GAME_BLACKJACK, &cfg, &info) == CS_E_UNSUPPORTED);
    cfg.num_players = 1;
    cfg.rng_mode = CS_RNG_PHILOX;
    EXPECT(cs_game_info_get(CS_GAME_BLACKJACK, &cfg, &info) == CS_E_UNSUPPORTED);
    cfg.rng_mode = CS_RNG_MT19937;
    cfg.num_decks = -1;
    cfg.num_players = 9;
    EXPECT(cs_game_info_get(CS_GAME_LEDUC, &cfg, &info) != CS_OK);
    EXPECT(strlen(cs_last_error()) > 0);
    cfg.num_players = 0;
    cs_handle* h = nullptr;
    EXPECT(cs_create(nullptr, CS_GAME_LEDUC, 4, 0, &cfg) == CS_E_INVALID);
    EXPECT(cs_create(&h, CS_GAME_LEDUC, 0, 0, &cfg) == CS_E_INVALID && h == nullptr);
    const int r = cs_create(&h, CS_GAME_LEDUC, 4, 0, &cfg);   // no GPU in the build container
    if (r == CS_OK) cs_destroy(h);
    else EXPECT(r == CS_E_DEVICE && h == nullptr && strlen(cs_last_error()) > 0);
    EXPECT(cs_seed(nullptr, nullptr, nullptr, 0, 1, nullptr) == CS_E_INVALID);
    EXPECT(cs_reset(nullptr, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_step(nullptr, nullptr, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_observe(nullptr, 0, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_rollout(nullptr, 1, 0, 0, 0, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_transitions(nullptr, 1, nullptr, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_legal_lists(nullptr, nullptr, 1, nullptr, nullptr, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_action_features(nullptr, nullptr, 1, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_cfr_train(nullptr, 1, 0, nullptr, nullptr, nullptr, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_get_env_state(nullptr, 0, nullptr, 0) == CS_E_INVALID);
    EXPECT(cs_set_env_state(nullptr, 0, nullptr, 0) == CS_E_INVALID);
    EXPECT(cs_get_rng_ctl(nullptr, 0, nullptr) == CS_E_INVALID);
    EXPECT(cs_copy_env_state(nullptr, 0, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_debug_holdem_rank7(nullptr, 1, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_debug_ddz_legal(nullptr, nullptr, nullptr, 1, nullptr, nullptr) == CS_E_INVALID);
    EXPECT(cs_debug_set_kernel_flags(nullptr, 0) == CS_E_INVALID);
    EXPECT(strlen(cs_version()) > 0);
    cs_destroy(nullptr);
}

int main()
{
    std::vector<uint8_t> host;
    size_t off[4];
    cs::ddz::Tab tab;
    memset(&tab, 0, sizeof(tab));
    const std::string err = cs::ddz::table_build_host(host, off, &tab);
    EXPECT(err.empty());
    EXPECT(tab.ng == 308 && tab.rocket > 0 && tab.bomb_hi > tab.bomb_lo);
    abi_host();
    if (!err.empty()) return 1;
    oracle_ddz_table(host, off);
    oracle_games();
    oracle_cfr_and_kats();
    printf("san_driver: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
