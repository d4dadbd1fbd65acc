/* Forced include for building the reference in oracle/_ref (container only).
 * my_compress.cpp:3732 (a startup self-print inside main(), not on the
 * compress path) calls abs() on a uInt32, which is ambiguous against
 * libstdc++'s overload set.  This one overload makes that line well-formed.
 * No header, library, tool or generated code of the reference is stubbed. */
#include <cstdlib>
inline unsigned int abs(unsigned int x) { return x; }
