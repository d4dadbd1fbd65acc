// fcx_match_rest.hip — k_match_rest: the general match kernel's tile body looped over the tiles of a
// routed call that no unit launch covered (fcx_match.hip, FCX_REST; fcx_route.hip).
#define FCX_REST 1
#define FCX_REST_WAVES 4   // looped, the body needs 128 VGPRs: at the 8-wave cap it spilled 149-185 of them
#include "fcx_match.hip"
