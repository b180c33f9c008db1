// hpmpc_api.h -- the public C ABI with default visibility.  The library is compiled with -fvisibility=hidden, so
// exactly the functions declared in include/hpmpc_mi355x.h are exported (a definition takes the visibility of
// its first declaration); the internal launch helpers and kernel stubs stay out of a caller's namespace.
#pragma once
#pragma GCC visibility push(default)
#include "../../include/hpmpc_mi355x.h"
#pragma GCC visibility pop
