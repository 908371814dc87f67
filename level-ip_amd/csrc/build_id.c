/* build_id.c — lvlip_build_id() (include/lvlip_csum.h): the SHA-256 (first 16
 * hex digits) of the product's sources, in the order level-ip_amd/BUILD_SOURCES
 * lists them, computed by level-ip_amd/Makefile at build time.  tests/conftest.py,
 * __graft_entry__.smoke() and bench.py compute the same hash over the tree
 * (lvlip.source_build_id) and refuse a library built from other sources. */
#include "lvlip_csum.h"

#ifndef LVLIP_BUILD_ID
#error "LVLIP_BUILD_ID is defined by level-ip_amd/Makefile"
#endif

const char *lvlip_build_id(void) { return LVLIP_BUILD_ID; }
