// cs_holdem_n22.hip -- Limit / No-limit hold'em with 17..22 players: cs_holdem_nrange.inc instantiated in its own
// translation unit (the units compile in parallel); reached through cs_holdem_n.hip's launchers.
#define CS_NP_LO 17
#define CS_NP_HI 22
#define CS_NP_NAME(x) np22_##x
#include "cs_holdem_nrange.inc"
