/*
 * tests/native/abi_layout.c -- compile-time check of include/kbz_plugin.h against the REFERENCE's
 * own instrumentation/instrumentation.h (built by tests/test_abi.py with
 * -I /root/reference/instrumentation; skipped where the reference is absent).
 *
 * Every member of kbz_instrumentation_t that the reference declares sits at the same offset and
 * has a type assignable to the reference member without a cast (-Werror), and the two appended
 * members start right where the reference struct ends, so a reference caller can copy the first
 * sizeof(instrumentation_t) bytes into its own instrumentation_t (instrumentation.h:40-62).
 */
#include <stddef.h>
#include <sys/types.h>
#define INSTRUMENTATION_NO_IMPORT
#include "instrumentation.h" /* the reference's header */
#include "kbz_plugin.h"

#define SAME_OFFSET(m)                                                                   \
  _Static_assert(offsetof(instrumentation_t, m) == offsetof(kbz_instrumentation_t, m), \
                 "offset of " #m)
SAME_OFFSET(create);
SAME_OFFSET(cleanup);
SAME_OFFSET(merge);
SAME_OFFSET(get_state);
SAME_OFFSET(free_state);
SAME_OFFSET(set_state);
SAME_OFFSET(enable);
SAME_OFFSET(is_new_path);
SAME_OFFSET(get_fuzz_result);
SAME_OFFSET(get_module_info);
SAME_OFFSET(get_edges);
SAME_OFFSET(is_process_done);
_Static_assert(offsetof(kbz_instrumentation_t, triage_batch) == sizeof(instrumentation_t),
               "triage_batch is appended right after the reference members");
_Static_assert(sizeof(kbz_instrumentation_edge_t) == sizeof(instrumentation_edge_t), "edge");
_Static_assert(offsetof(kbz_instrumentation_edges_t, edges) ==
                   offsetof(instrumentation_edges_t, edges), "edges");

int main(void) {
  kbz_instrumentation_t k = {0};
  instrumentation_t r;
  /* member types: each assignment must compile without a cast under -Werror */
  r.create = k.create;
  r.cleanup = k.cleanup;
  r.merge = k.merge;
  r.get_state = k.get_state;
  r.free_state = k.free_state;
  r.set_state = k.set_state;
  r.enable = k.enable;
  r.is_new_path = k.is_new_path;
  r.get_fuzz_result = k.get_fuzz_result;
  r.get_module_info = k.get_module_info;
  r.get_edges = (instrumentation_edges_t * (*)(void *, int))k.get_edges; /* struct tag differs */
  r.is_process_done = k.is_process_done;
  return r.create != NULL;
}
