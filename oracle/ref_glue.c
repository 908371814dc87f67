/*
 * oracle/ref_glue.c — the one symbol level-ip's src/main.c exports to the rest
 * of the stack (`running`, read by the worker loops, e.g. src/netdev.c:88).
 * Linked into oracle/_ref/libref.so so the reference objects resolve without
 * main.c (which needs libcap).  Test infrastructure only.
 */
int running = 1;
