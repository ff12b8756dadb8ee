/*
 * or_cfr.c -- TEST INFRASTRUCTURE ONLY (see oracle.h). Scalar restatement of the reference's chance-sampling CFR
 * agent on Leduc Hold'em, over the oracle's Leduc game (or_leduc.c).
 *
 * Follows rlcard/agents/cfr_agent.py:
 *   :30-43   train: iteration += 1; per player: env.reset() (a new deal from the env's RandomState), traverse_tree
 *            with reach probabilities [1, 1]; then update_policy
 *   :45-98   traverse_tree: terminal -> env.get_payoffs(); else for each legal action (ascending): reach of the
 *            acting player *= action prob, env.step / recurse / env.step_back; state utility += prob * utility; at the
 *            traversing player's nodes regrets[obs][a] += cf_prob * (u_a - u) and average_policy[obs][a] +=
 *            iteration * player_prob * action_prob
 *   :100-123 update_policy / regret_matching (positive part / positive sum, else 1 / num_actions)
 *   :125-146 action_probs: unseen obs -> uniform 1 / num_actions (and inserted into policy), then
 *            utils/utils.py:181-198 remove_illegal (zero illegal, uniform if the sum is 0, else divide by the sum)
 * The infoset key (the float64 obs bytes of envs/leducholdem.py:41-71) is held as its index in the dense table:
 *   ((hand * 4 + public + 1 (0 = none)) * 15 + my_chips) * 15 + others' chips   (OR_CFR_INFOSETS = 2700 rows).
 * Every floating-point operation is done in the reference's order (no contraction), so results are bit-exact.
 * Generalisation used by the GPU engine's batched mode: n envs, each dealing its own game per player per iteration
 * (players outer, envs inner); n = 1 is the reference agent.
 */
#include <stdlib.h>
#include <string.h>
#include "or_games.h"


#define NA 4
#define MAXD 16

struct or_cfr {
    int64_t n;
    or_mt *rng;
    uint8_t *envs;       /* n Leduc env blobs (the game each env holds after its last deal) */
    size_t esz;
    int64_t iteration;
    double policy[OR_CFR_INFOSETS][NA], avg[OR_CFR_INFOSETS][NA], regrets[OR_CFR_INFOSETS][NA];
    uint8_t flags[OR_CFR_INFOSETS];   /* bit 0: key in policy, bit 1: key in regrets / average_policy */
};

int or_cfr_infoset(const uint8_t *obs)
{
    int h = -1, pub = 0, my = -1, op = -1;
    for (int i = 0; i < 3; i++) if (obs[i]) h = i;
    for (int i = 0; i < 3; i++) if (obs[3 + i]) pub = i + 1;
    for (int i = 0; i < 15; i++) if (obs[6 + i]) my = i;
    for (int i = 0; i < 15; i++) if (obs[21 + i]) op = i;
    if (h < 0 || my < 0 || op < 0) return -1;
    return ((h * 4 + pub) * 15 + my) * 15 + op;
}

static const or_game_vt *VT = &or_leduc_vt;

static void action_probs(or_cfr *c, int idx, unsigned legal, double out[NA])
{
    double row[NA];
    if (!(c->flags[idx] & 1)) {                     /* unseen: uniform, inserted into self.policy */
        for (int a = 0; a < NA; a++) c->policy[idx][a] = 1.0 / NA;
        c->flags[idx] |= 1;
    }
    for (int a = 0; a < NA; a++) row[a] = c->policy[idx][a];
    double p[NA] = {0, 0, 0, 0};
    int nl = 0;
    for (int a = 0; a < NA; a++) if (legal >> a & 1) { p[a] = row[a]; nl++; }
    double s = 0.0;
    for (int a = 0; a < NA; a++) s = s + p[a];
    if (s == 0.0) {
        for (int a = 0; a < NA; a++) if (legal >> a & 1) p[a] = 1.0 / (double)nl;
    } else {
        for (int a = 0; a < NA; a++) p[a] = p[a] / s;
    }
    memcpy(out, p, sizeof(p));
}

/* traverse_tree on the env blob `e` (restored by the caller after return, = step_back); returns utilities */
static void traverse(or_cfr *c, uint8_t *e, const double probs[2], int player, double util[2], int depth)
{
    if (VT->is_over(e)) {
        float r[2];
        VT->payoffs(e, NULL, r);
        util[0] = (double)r[0];
        util[1] = (double)r[1];
        return;
    }
    const int cp = VT->current_player(e);
    uint8_t obs[36], lb[1] = {0};
    VT->observe(e, cp, obs, lb);
    const int idx = or_cfr_infoset(obs);
    const unsigned legal = lb[0];
    double ap[NA];
    action_probs(c, idx, legal, ap);
    double su[2] = {0.0, 0.0}, au[NA] = {0, 0, 0, 0};
    uint8_t *child = (uint8_t *)malloc(c->esz);
    for (int a = 0; a < NA; a++) {
        if (!(legal >> a & 1)) continue;
        double np_[2] = {probs[0], probs[1]};
        np_[cp] = np_[cp] * ap[a];
        memcpy(child, e, c->esz);
        VT->step(child, NULL, a);
        double u[2];
        traverse(c, child, np_, player, u, depth + 1);
        su[0] = su[0] + ap[a] * u[0];
        su[1] = su[1] + ap[a] * u[1];
        au[a] = u[cp];
    }
    free(child);
    if (cp == player) {
        const double pp = probs[cp];
        const double cf = cp == 0 ? 1.0 * probs[1] : probs[0] * 1.0;
        c->flags[idx] |= 2;
        for (int a = 0; a < NA; a++) {
            if (!(legal >> a & 1)) continue;
            const double regret = cf * (au[a] - su[cp]);
            c->regrets[idx][a] = c->regrets[idx][a] + regret;
            c->avg[idx][a] = c->avg[idx][a] + ((double)c->iteration * pp) * ap[a];
        }
    }
    util[0] = su[0];
    util[1] = su[1];
}

or_cfr *or_cfr_create(int64_t n, const uint32_t *keys, const int32_t *key_len)
{
    or_cfr *c = (or_cfr *)calloc(1, sizeof(or_cfr));
    or_cfg cfg = {2, 0, 100, -1, 0};
    c->n = n;
    c->esz = (VT->env_size(&cfg) + 15) & ~(size_t)15;
    c->envs = (uint8_t *)calloc((size_t)n, c->esz);
    c->rng = (or_mt *)calloc((size_t)n, sizeof(or_mt));
    for (int64_t i = 0; i < n; i++) or_mt_seed_by_array(&c->rng[i], keys + 2 * i, key_len[i]);
    return c;
}

void or_cfr_destroy(or_cfr *c)
{
    if (!c) return;
    free(c->envs);
    free(c->rng);
    free(c);
}

void or_cfr_train(or_cfr *c, int32_t iterations)
{
    or_cfg cfg = {2, 0, 100, -1, 0};
    for (int32_t it = 0; it < iterations; it++) {
        c->iteration += 1;
        for (int p = 0; p < 2; p++) {
            for (int64_t i = 0; i < c->n; i++) {
                uint8_t *e = c->envs + (size_t)i * c->esz;
                VT->init_game(e, &c->rng[i], &cfg);
                const double probs[2] = {1.0, 1.0};
                double u[2];
                traverse(c, e, probs, p, u, 0);
            }
        }
        for (int k = 0; k < OR_CFR_INFOSETS; k++) {     /* update_policy: every key of regrets */
            if (!(c->flags[k] & 2)) continue;
            double pos = 0.0;
            for (int a = 0; a < NA; a++) if (c->regrets[k][a] > 0) pos = pos + c->regrets[k][a];
            for (int a = 0; a < NA; a++) {
                if (pos > 0) {
                    const double x = c->regrets[k][a] / pos;
                    c->policy[k][a] = x > 0.0 ? x : 0.0;
                } else {
                    c->policy[k][a] = 1.0 / NA;
                }
            }
            c->flags[k] |= 1;
        }
    }
}

void or_cfr_tables(const or_cfr *c, double *policy, double *avg, double *regrets, uint8_t *flags)
{
    memcpy(policy, c->policy, sizeof(c->policy));
    memcpy(avg, c->avg, sizeof(c->avg));
    memcpy(regrets, c->regrets, sizeof(c->regrets));
    memcpy(flags, c->flags, sizeof(c->flags));
}

uint64_t or_cfr_draws(const or_cfr *c, int64_t env) { return c->rng[env].ndraw; }
