// cs_prof.h -- PROFILING BUILDS ONLY. Each macro below, set on an A/B build (`make variant NAME=x
// DEFS=-DCS_PROF_NO_OBS=1`), drops one piece of a kernel so that its share of the launch time can be measured. Such a
// build's outputs are WRONG: it is never the product library (libcardsim.so is built with every macro at 0), and
// bench.py marks a line measured on any other library as a non-product build. The measured splits are in DESIGN.md and
// profiles/EXPERIMENTS.md.
#pragma once

#ifndef CS_PROF_NO_OBS
#define CS_PROF_NO_OBS 0       // k_rollout (cs_skeleton.h): no obs rows
#endif
#ifndef CS_PROF_NO_SMALL
#define CS_PROF_NO_SMALL 0     // k_rollout: no legal / player / reward / done rows
#endif
#ifndef CS_PROF_NO_RESET
#define CS_PROF_NO_RESET 0     // Leduc: no deal at a reset (wrong deals)
#endif
#ifndef CS_PROF_NO_EVAL
#define CS_PROF_NO_EVAL 0      // Limit / No-limit: no showdown evaluator
#endif
#ifndef CS_PROF_NO_DEAL9
#define CS_PROF_NO_DEAL9 0     // Limit / No-limit: no tracked draws of the nine dealt positions
#endif
#ifndef CS_PROF_NO_TRACK
#define CS_PROF_NO_TRACK 0     // Limit / No-limit: no swap trace-back of the dealt cards
#endif
#ifndef CS_PROF_NO_SKIP
#define CS_PROF_NO_SKIP 0      // Limit / No-limit: no skip scan of the 42 undealt draws
#endif
#ifndef CS_PROF_DDZ
#define CS_PROF_DDZ 0          // DouDizhu k_rollout2: bit 0 no legal rows, bit 1 no obs rows
#endif
