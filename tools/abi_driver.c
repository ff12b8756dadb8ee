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
    or_cfg oc = {info.num_players, 1};
    or_batch* b = or_batch_create(game, W, &oc);
    or_batch_seed(b, keys, klen);
    size_t wr = (size_t)T * W;
    uint8_t* eo = calloc(wr, info.obs_dim);
    uint8_t* el = calloc(wr, info.legal_bytes);
    uint8_t* ep = calloc(wr, 1);
    int32_t* ea = calloc(wr, 4);
    float* er = calloc(wr * info.num_players, 4);
    uint8_t* ed = calloc(wr, 1);
    uint8_t* tmp_o = calloc(W, info.obs_dim);
    uint8_t* tmp_l = calloc(W, info.legal_bytes);
    uint8_t* tmp_p = calloc(W, 1);
    float* tmp_r = calloc(W * info.num_players, 4);
    uint8_t* tmp_d = calloc(W, 1);
    or_batch_reset(b, tmp_o, tmp_l, tmp_p, tmp_r, tmp_d);
    or_batch_rollout(b, T, 5, 0, 0, eo, el, ep, ea, er, ed, NULL);
    long long bad = 0;
    for (int t = 0; t < T; t++)
        for (long long i = 0; i < W; i++) {
            size_t g = (size_t)t * n + i, e = (size_t)t * W + i;
            int a = info.action_bytes == 1 ? ((uint8_t*)host[3])[g] : ((int16_t*)host[3])[g];
            if (memcmp((uint8_t*)host[0] + g * info.obs_dim, eo + e * info.obs_dim, info.obs_dim) ||
                memcmp((uint8_t*)host[1] + g * info.legal_bytes, el + e * info.legal_bytes, info.legal_bytes) ||
                ((uint8_t*)host[2])[g] != ep[e] || a != ea[e] || ((uint8_t*)host[5])[g] != ed[e] ||
                memcmp((float*)host[4] + g * info.num_players, er + e * info.num_players, 4 * info.num_players)) {
                if (bad < 5) fprintf(stderr, "mismatch t=%d env=%lld\n", t, i);
                bad++;
            }
        }
    printf("parity: %lld mismatching rows of %lld\n", bad, (long long)T * W);
    cs_destroy(h);
    return bad ? 6 : 0;
}
