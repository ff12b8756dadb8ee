// cs_holdem_n10.hip -- Limit / No-limit hold'em with 7..10 players: cs_holdem_nrange.inc instantiated in its own
// translation unit (the units compile in parallel); reached through cs_holdem_n.hip's launchers.
#define CS_NP_LO 7
#define CS_NP_HI 10
#define CS_NP_NAME(x) np10_##x
#include "cs_holdem_nrange.inc"
