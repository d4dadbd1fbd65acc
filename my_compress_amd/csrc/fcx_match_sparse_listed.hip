// fcx_match_sparse_listed.hip — the sparse unit's listed kernel instance (k_match<false, true>: its tiles from
// the unit's list in a routed call, fcx_route.hip).  Its own translation unit: beside the direct
// instance it moved that kernel's code (fcx_match.hip FCX_LISTED).
#define FCX_SPARSE 1
#define FCX_LISTED 1
#include "fcx_match.hip"
