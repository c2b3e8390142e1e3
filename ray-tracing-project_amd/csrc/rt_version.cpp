// rt_version.cpp -- ties a built librtamd.so to the sources it was built from: the Makefile hashes
// every product source (csrc/*.hip, *.cpp, *.h and include/rt/rt_api.h, concatenated in sorted path
// order, SHA-256, first 16 hex digits) into build/rt_version.h; tools and tests recompute the same
// hash over the tree they run from (rtamd.source_hash()) and compare (bench line "build", smoke()).
#include "../../include/rt/rt_api.h"
#include "rt_version.h"  // generated: RT_SOURCE_HASH

#define RT_VERSION_STR2(x) #x
#define RT_VERSION_STR(x) RT_VERSION_STR2(x)

extern "C" const char* rt_version_string(void) {
  return "librtamd api " RT_VERSION_STR(RT_API_VERSION) " gfx950 sources " RT_SOURCE_HASH;
}
extern "C" const char* rt_source_hash(void) { return RT_SOURCE_HASH; }
