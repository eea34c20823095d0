// engine_internal.h -- the fused engine's pieces fh_dgraph reuses (engine.hip).
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "fh_common.h"
#include "scan.h"

namespace fh {

struct EngineDevice;
EngineDevice *engine_new(const fh_config &cfg);
void engine_free(EngineDevice *e);
// element logs holding a subset of the batch's positions (one key shard's
// processes); runs then compute KeyDeps only
void engine_stage_subset(EngineDevice *e, const fh_stream_desc &d, const uint64_t *dot,
                         const uint64_t *key, const uint64_t *off, const uint32_t *ent);
// rewind + KeyDeps over the staged logs: the u32 dependency code of every
// staged position (0 none, vid + 1, or 0x80000000 | log position)
const uint32_t *engine_run_codes(EngineDevice *e, float *ms);
hipStream_t engine_stream(EngineDevice *e);
void engine_set_profiling(EngineDevice *e, bool on);
std::vector<std::pair<std::string, float>> engine_times(EngineDevice *e);

// The QuorumDeps / MShardCommit union over n commands of S codes each (codes
// vid + 1 or 0; vids index `dot`): committed deps as CSR of ascending dots
// (dep_off[n+1], dep_dot), graph edges at dst[i*S ..) (vids, padded with
// vbase + i) and their counts ecnt[n].  scal: 2 scratch words.
void union_rows(uint32_t n, uint32_t S, const uint32_t *codes, const uint64_t *dot,
                uint32_t vbase, uint32_t *dcnt, uint32_t *dep_off, uint64_t *dep_dot,
                uint32_t *dst, uint32_t *ecnt, uint32_t *scal, ScanWorkspace &ws, hipStream_t s);

}  // namespace fh
