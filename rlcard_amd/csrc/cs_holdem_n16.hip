// cs_holdem_n16.hip -- Limit / No-limit hold'em with 11..16 players: cs_holdem_nrange.inc instantiated in its own
// translation unit (the units compile in parallel); reached through cs_holdem_n.hip's launchers.
#define CS_NP_LO 11
#define CS_NP_HI 16
#define CS_NP_NAME(x) np16_##x
#include "cs_holdem_nrange.inc"
