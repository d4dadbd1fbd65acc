// fcx_match_rest_runs.hip — k_match_rest_runs: the runs unit's tile body looped over the entries of its list
// that no launch of the unit covered in a routed call (fcx_match.hip FCX_REST, fcx_route.hip).  Its own
// translation unit: the unit's k_match keeps its code generation.
#define FCX_RUNS 1
#define FCX_NOBUCKET 1
#define FCX_REST 1
#define FCX_REST_WAVES 4   // looped, the body needs up to 128 VGPRs (at the 8-wave cap: 22-95 spilled)
#include "fcx_match.hip"
