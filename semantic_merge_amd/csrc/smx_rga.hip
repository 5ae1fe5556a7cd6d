// smx_rga.hip — batched RGA replay (semmerge/crdt.py:23-57).  (in progress)
#include "smx_common.h"

extern "C" int smx_rga_workspace_bytes(int64_t n_ops, int64_t n_lists, size_t* bytes) {
  if (!bytes) return SMX_E_ARG;
  *bytes = 0;
  (void)n_ops;
  (void)n_lists;
  return SMX_E_ARG;
}

extern "C" int smx_rga_replay(const smx_rga_ops* ops, const smx_rga_out* out, void* ws, size_t wsb,
                              void* stream) {
  (void)ops; (void)out; (void)ws; (void)wsb; (void)stream;
  return SMX_E_ARG;
}
