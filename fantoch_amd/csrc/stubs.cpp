// stubs.cpp -- temporary FH_ENOTIMPL entry points (replaced as subsystems land).
#include "fh_common.h"

#define STUB(sig) \
  sig { fh::set_last_error("not implemented yet"); return FH_ENOTIMPL; }

extern "C" {
STUB(fh_status fh_graph_create(uint32_t, uint64_t, const fh_config *, fh_graph **))
STUB(fh_status fh_graph_destroy(fh_graph *))
STUB(fh_status fh_graph_add_batch(fh_graph *, size_t, const uint64_t *, const uint32_t *,
                                  const uint64_t *, const uint32_t *, const uint64_t *))
STUB(fh_status fh_graph_drain(fh_graph *, uint64_t *, uint64_t *, size_t, size_t *))
STUB(fh_status fh_graph_mark_executed(fh_graph *, size_t, const uint64_t *))
STUB(fh_status fh_graph_set_executed_frontier(fh_graph *, uint32_t, uint64_t))
STUB(fh_status fh_graph_pending(fh_graph *, size_t *))
STUB(fh_status fh_graph_missing(fh_graph *, uint64_t *, size_t, size_t *))
}
