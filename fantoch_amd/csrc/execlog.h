// execlog.h -- a parsed execution log (execlog.cpp), one event per
// GraphExecutionInfo entry in log order.  Shared with graph_api.hip, whose
// fh_execlog_replay feeds the events to an fh_graph.
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "fh_common.h"

namespace fh {

struct ExecLog {
  uint64_t shard_id = 0;  // Command::keys(shard_id) become the events' keys
  // per event: FH_LOG_* kind; dot (Add / Info / reply Executed); the
  // command's rifl; shards = Command::shards() mask (Add / Info) or the
  // requesting shard (Request); Dependency dots + shard masks (Add / Info),
  // or the dots of a Request / Executed
  std::vector<uint8_t> kind;
  std::vector<uint64_t> dot, rifl_client, rifl_seq, shards;
  std::vector<uint8_t> read_only;
  std::vector<uint32_t> key_off{0}, dep_off{0};
  std::vector<uint64_t> key_id, dep_dot, dep_shards;
  std::vector<std::string> key_names;  // interned in first-seen order
  std::unordered_map<std::string, uint64_t> key_ids;
  size_t frames = 0;
};

void parse_execlog(ExecLog &log, const uint8_t *buf, size_t len);
const ExecLog &execlog_of(const fh_execlog *h);

}  // namespace fh
