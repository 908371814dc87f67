/* stamp.c — the build stamp of the lab and testkit libraries
 * (lvlip_lab_build_id / lvlip_testkit_build_id): the SHA-256 (first 16 hex
 * digits) of the files level-ip_amd/LAB_SOURCES / TESTKIT_SOURCES list,
 * computed by level-ip_amd/Makefile.  lvlip.lab() and lvlip.testkit() refuse
 * a library whose stamp differs from the tree's, as lvlip refuses a stale
 * product (build_id.c). */
#if !defined(LVLIP_STAMP_FN) || !defined(LVLIP_STAMP)
#error "LVLIP_STAMP_FN and LVLIP_STAMP are defined by level-ip_amd/Makefile"
#endif

__attribute__((visibility("default"))) const char *LVLIP_STAMP_FN(void) { return LVLIP_STAMP; }
