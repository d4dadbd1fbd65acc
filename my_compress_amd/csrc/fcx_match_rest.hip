// fcx_match_rest.hip — k_match_rest: the general match kernel's tile body looped over the tiles of a
// routed call that no unit launch covered (fcx_match.hip, FCX_REST; fcx_route.hip).
#define FCX_REST 1
#include "fcx_match.hip"
