// fcx_match_nf_direct.hip — the nf unit's checked direct kernel instance (k_match<false, false, true>: every tile
// of the grid, those of other kinds ending at their kind byte; fcx_route.hip).  Its own translation unit:
// beside the unrouted instances it moved their code (fcx_match.hip FCX_DIRECT).
#define FCX_NOFILTER 1
#define FCX_UNIT_ILP 2
#define FCX_DIRECT 1
#include "fcx_match.hip"
