/*
 * abi_driver.c -- native (no Python, no torch) exercise of the C ABI against the CPU oracle.
 * Test/diagnostic tool: links rlcard_amd/libcardsim.so (product) and oracle/liboracle.so (checker).
 *
 *   abi_driver <game_id> <num_envs> <T> [window]
 * Seeds env i with the key of seed 42+i (keys computed by the caller-side helper below from a precomputed table
 * file is overkill here: we take the keys from stdin as "k0 k1 len" lines), resets, runs one rollout of T steps,
 * copies back, and compares the first `window` envs bit-exactly against the oracle.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../include/cardsim.h"
#include "../oracle/oracle.h"

/* Draws that env's queued deals consumed, decoded from its cs_get_env_state words with nothing but the layout
 * include/cardsim.h documents at cs_get_env_state (header word after game_words, CB = log2(DQ) + 1, XB = 2 CB - 1,
 * per slot 7 low draw bits in e0 bits 25..31 and 2 high bits in the header at XB + 2 + 2 slot). */
static uint32_t queued_draws(const uint32_t* w, const cs_game_info* info)
{
    const uint32_t dq = (uint32_t)info->deal_queue_depth;
    if (dq == 0) return 0;
    uint32_t cb = 1;
    while ((1u << (cb - 1)) < dq) cb++;                 /* log2(DQ) + 1 */
    const uint32_t xb = 2 * cb - 1, hdr = w[info->game_words];
    const uint32_t count = hdr & ((1u << cb) - 1u), head = (hdr >> cb) & (dq - 1u);
    uint32_t d = 0;
    for (uint32_t i = 0; i < count; i++) {
        const uint32_t slot = (head + i) % dq;
        d += ((w[info->game_words + 1 + 2 * slot] >> 25) & 127u) | ((hdr >> (xb + 2 + 2 * slot)) & 3u) << 7;
    }
    return d;
}

#define CHECK(x)                                                                 \
    do {                                                                         \
        int rc_ = (x);                                                           \
        if (rc_ != 0) {                                                          \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, cs_last_error());     \
            return 2;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: abi_driver game n T [window] < keys\n");
        return 1;
    }
    int game = atoi(argv[1]);
    long long n = atoll(argv[2]);
    int T = atoi(argv[3]);
    long long W = argc > 4 ? atoll(argv[4]) : (n < 512 ? n : 512);
    uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * 2 * n);
    int32_t* klen = (int32_t*)malloc(sizeof(int32_t) * n);
    for (long long i = 0; i < n; i++) {
        unsigned a, b;
        int l;
        if (scanf("%u %u %d", &a, &b, &l) != 3) {
            fprintf(stderr, "short key input at %lld\n", i);
            return 1;
        }
        keys[2 * i] = a;
        keys[2 * i + 1] = b;
        klen[i] = l;
    }
    if (cs_abi_version() < CS_ABI_VERSION) {   /* cs_game_info of this header's size (include/cardsim.h) */
        fprintf(stderr, "library ABI %d < header ABI %d\n", (int)cs_abi_version(), CS_ABI_VERSION);
        return 2;
    }
    cs_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.num_decks = -1;
    cs_game_info info;
    CHECK(cs_game_info_get(game, &cfg, &info));
    cs_handle* h = NULL;
    CHECK(cs_create(&h, game, n, 0, &cfg));
    CHECK(cs_seed(h, keys, klen, 0, n, NULL));
    printf("seed ok\n");
    fflush(stdout);
    cs_traj_out o;
    size_t rows = (size_t)T * n;
    size_t sz[6] = {rows * info.obs_dim, rows * info.legal_bytes, rows, rows * info.action_bytes,
                    rows * info.num_players * 4, rows};
    void* dev[6];
    for (int k = 0; k < 6; k++)
        if (hipMalloc(&dev[k], sz[k]) != hipSuccess) return 3;
    o.obs = dev[0]; o.legal = dev[1]; o.player = dev[2]; o.action = dev[3]; o.reward = dev[4]; o.done = dev[5];
    o.final_obs = NULL;
    cs_step_out so;
    memset(&so, 0, sizeof(so));
    CHECK(cs_reset(h, &so, NULL));
    CHECK(cs_rollout(h, T, 5, 0, 0, &o, NULL));
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "rollout failed: %s\n", hipGetErrorString(hipGetLastError()));
        return 4;
    }
    printf("rollout ok\n");
    void* host[6];
    for (int k = 0; k < 6; k++) {
        host[k] = malloc(sz[k]);
        if (hipMemcpy(host[k], dev[k], sz[k], hipMemcpyDeviceToHost) != hipSuccess) return 5;
    }
    /* oracle on the first W envs */
    or_cfg oc = {info.num_players, 1, 100, -1, 0};   /* the cs_config defaults: 1 deck, 100 chips, dealer drawn */
    or_batch* b = or_batch_create(game, W, &oc);
    or_batch_seed(b, keys, klen);
    size_t wr = (size_t)T * W;
    uint8_t* eo = (uint8_t*)calloc(wr, info.obs_dim);
    uint8_t* el = (uint8_t*)calloc(wr, info.legal_bytes);
    uint8_t* ep = (uint8_t*)calloc(wr, 1);
    int32_t* ea = (int32_t*)calloc(wr, 4);
    float* er = (float*)calloc(wr * info.num_players, 4);
    uint8_t* ed = (uint8_t*)calloc(wr, 1);
    uint8_t* tmp_o = (uint8_t*)calloc(W, info.obs_dim);
    uint8_t* tmp_l = (uint8_t*)calloc(W, info.legal_bytes);
    uint8_t* tmp_p = (uint8_t*)calloc(W, 1);
    float* tmp_r = (float*)calloc(W * info.num_players, 4);
    uint8_t* tmp_d = (uint8_t*)calloc(W, 1);
    or_batch_reset(b, tmp_o, tmp_l, tmp_p, tmp_r, tmp_d);
    or_batch_rollout(b, T, 5, 0, 0, eo, el, ep, ea, er, ed, NULL);
    long long bad = 0;
    for (int t = 0; t < T; t++)
        for (long long i = 0; i < W; i++) {
            size_t g = (size_t)t * n + i, e = (size_t)t * W + i;
            int a = info.action_bytes == 1 ? ((uint8_t*)host[3])[g] : ((int16_t*)host[3])[g];
            const char* what = NULL;
            if (memcmp((uint8_t*)host[0] + g * info.obs_dim, eo + e * info.obs_dim, info.obs_dim)) what = "obs";
            else if (memcmp((uint8_t*)host[1] + g * info.legal_bytes, el + e * info.legal_bytes, info.legal_bytes))
                what = "legal";
            else if (((uint8_t*)host[2])[g] != ep[e]) what = "player";
            else if (a != ea[e]) what = "action";
            else if (((uint8_t*)host[5])[g] != ed[e]) what = "done";
            else
                for (int k = 0; k < info.num_players; k++)   /* by value, as the Python tests (numpy) compare */
                    if (((float*)host[4])[g * info.num_players + k] != er[e * info.num_players + k]) what = "reward";
            if (what) {
                if (bad < 5) fprintf(stderr, "mismatch t=%d env=%lld: %s\n", t, i, what);
                bad++;
            }
        }
    printf("parity: %lld mismatching rows of %lld\n", bad, (long long)T * W);
    /* stream position of every checked env's current game: ctl position minus its queued deals' draws (header-only
     * decode) against the oracle's draws, which never draws ahead */
    long long badpos = 0, queued = 0;
    if (info.state_words != info.game_words + (info.deal_queue_depth ? 1 + 2 * info.deal_queue_depth : 0)) {
        fprintf(stderr, "state_words %d != game_words %d + queue of %d\n", info.state_words, info.game_words,
                info.deal_queue_depth);
        return 7;
    }
    uint32_t* words = (uint32_t*)malloc(sizeof(uint32_t) * info.state_words);
    for (long long i = 0; i < W; i++) {
        uint32_t ctl;
        CHECK(cs_get_env_state(h, i, words, info.state_words));
        CHECK(cs_get_rng_ctl(h, i, &ctl));
        const uint32_t q = queued_draws(words, &info);
        queued += q != 0;
        const uint32_t pos = ((ctl & (game == CS_GAME_DOUDIZHU ? 0x7FFu : 0x3FFFu)) + (uint32_t)info.rng_period - q) %
                             (uint32_t)info.rng_period;
        if (pos != (uint32_t)(or_batch_draws(b, i) % (uint64_t)info.rng_period)) {
            if (badpos < 5) fprintf(stderr, "stream position env=%lld: %u vs oracle %llu\n", i, pos,
                                    (unsigned long long)(or_batch_draws(b, i) % (uint64_t)info.rng_period));
            badpos++;
        }
    }
    printf("deal queue depth %d: %lld of %lld envs hold queued deals; stream positions: %lld mismatching\n",
           info.deal_queue_depth, queued, W, badpos);
    bad += badpos;
    cs_destroy(h);
    return bad ? 6 : 0;
}
