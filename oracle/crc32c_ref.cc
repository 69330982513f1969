// ORACLE TEST INFRASTRUCTURE -- a C entry point to the reference's own
// crc32c::Value (src/util/crc32c.h:19-21, crc32c.cc:292-335), which
// oracle/Makefile compiles in place from /root/reference together with this
// shim.  KEY_CACHING's signature is crc32c::Value of the first
// min(bytes, 2048) key bytes (key_caching.h:18,43).
#include <stddef.h>
#include <stdint.h>

#include "util/crc32c.h"

extern "C" uint32_t ref_crc32c(const char* p, size_t n) { return PS::crc32c::Value(p, n); }
