// execlog.cpp -- execution-log ingest.
//
// fantoch's runner can log every GraphExecutionInfo an executor receives
// (run/task/execution_logger.rs:11-55): each value is bincode-serialised
// (bincode 1.3 `bincode::serialize`: little-endian, fixed-width integers, u32
// enum variant index, u64 sequence/map/string lengths, u8 Option/bool tags;
// run/rw/mod.rs:87-100) and framed by tokio's LengthDelimitedCodec defaults (a
// 4-byte big-endian length before every frame, run/rw/mod.rs:20-36).  The
// replay binary (fantoch_ps/src/bin/graph_executor_replay.rs:13-38) feeds the
// frames to a GraphExecutor one by one; fh_execlog_replay feeds them to an
// fh_graph in batches.
//
// Serde layouts (derive order = field order):
//   GraphExecutionInfo  executor/graph/executor.rs:204-222
//     0 Add{dot: Dot, cmd: Command, deps: HashSet<Dependency>}
//     1 Request{from: ShardId, dots: HashSet<Dot>}
//     2 RequestReply{infos: Vec<RequestReply>}
//     3 Executed{dots: HashSet<Dot>}
//   RequestReply        executor/graph/mod.rs:33-43
//     0 Info{dot, cmd, deps: Vec<Dependency>}   1 Executed{dot}
//   Dot = Id<u8>{source: u8, sequence: u64}, Rifl = Id<u64>  fantoch/src/id.rs:7-27
//   Command{rifl, shard_to_ops: HashMap<ShardId, HashMap<Key, KVOp>>,
//           read_only: bool, _empty_keys: HashMap<Key, KVOp>}  command.rs:11-20
//   KVOp: 0 Get, 1 Put(String), 2 Delete                      kvs.rs:12-16
//   Dependency{dot, shards: Option<BTreeSet<ShardId>>}         deps/keys/mod.rs:18-22
#include <cstring>

#include "execlog.h"

namespace fh {

namespace {

struct Reader {
  const uint8_t *p, *end;
  size_t frame;
  const uint8_t *base;
  [[noreturn]] void fail(const char *what) const {
    throw Error(FH_EINVAL, "execution log frame " + std::to_string(frame) + " at byte " +
                               std::to_string(size_t(p - base)) + ": " + what);
  }
  void need(size_t n) const {
    if (size_t(end - p) < n) fail("truncated value");
  }
  uint8_t u8() {
    need(1);
    return *p++;
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t u64() {
    need(8);
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  bool boolean() {
    const uint8_t b = u8();
    if (b > 1) fail("invalid bool");
    return b;
  }
  uint64_t len() {
    const uint64_t n = u64();
    if (n > uint64_t(end - p)) fail("length exceeds frame");
    return n;
  }
  std::string string() {
    const uint64_t n = len();
    std::string s(reinterpret_cast<const char *>(p), size_t(n));
    p += n;
    return s;
  }
  uint64_t dot() {
    const uint8_t src = u8();
    const uint64_t seq = u64();
    if (src == 0) fail("dot with ProcessId 0");
    if (seq >> 56) fail("dot sequence >= 2^56 does not pack");
    return (uint64_t(src) << 56) | seq;
  }
};

struct Parser {
  ExecLog &log;
  Reader r;

  uint64_t intern(const std::string &k) {
    auto it = log.key_ids.find(k);
    if (it != log.key_ids.end()) return it->second;
    const uint64_t id = log.key_names.size();
    log.key_names.push_back(k);
    log.key_ids.emplace(k, id);
    return id;
  }

  void kvop() {
    switch (r.u32()) {
      case 0: break;              // Get
      case 1: (void)r.string(); break;  // Put(Value)
      case 2: break;              // Delete
      default: r.fail("invalid KVOp variant");
    }
  }

  // Command: keys of this shard (Command::keys, command.rs:95-100) go to the
  // event's key list; its shard set (Command::shards) becomes a bitmask.
  void command(uint64_t &client, uint64_t &seq, uint64_t &mask, uint8_t &ro) {
    client = r.u64();
    seq = r.u64();
    mask = 0;
    const uint64_t nshards = r.len();
    for (uint64_t s = 0; s < nshards; s++) {
      const uint64_t shard = r.u64();
      if (shard >= 64) r.fail("shard id >= 64 (shard sets are 64-bit masks)");
      mask |= uint64_t(1) << shard;
      const uint64_t nops = r.len();
      for (uint64_t o = 0; o < nops; o++) {
        std::string key = r.string();
        kvop();
        if (shard == log.shard_id) log.key_id.push_back(intern(key));
      }
    }
    ro = r.boolean();
    const uint64_t nempty = r.len();  // _empty_keys
    for (uint64_t o = 0; o < nempty; o++) {
      (void)r.string();
      kvop();
    }
  }

  void dependency() {
    log.dep_dot.push_back(r.dot());
    uint64_t mask = 0;
    switch (r.u8()) {
      case 0: break;  // None: a noop
      case 1: {
        const uint64_t n = r.len();
        for (uint64_t i = 0; i < n; i++) {
          const uint64_t s = r.u64();
          if (s >= 64) r.fail("shard id >= 64 (shard sets are 64-bit masks)");
          mask |= uint64_t(1) << s;
        }
        if (mask == 0) r.fail("empty shard set");
        break;
      }
      default: r.fail("invalid Option tag");
    }
    log.dep_shards.push_back(mask);
  }

  void close_event(uint8_t kind, uint64_t dot, uint64_t client, uint64_t seq, uint64_t shards,
                   uint8_t ro) {
    log.kind.push_back(kind);
    log.dot.push_back(dot);
    log.rifl_client.push_back(client);
    log.rifl_seq.push_back(seq);
    log.shards.push_back(shards);
    log.read_only.push_back(ro);
    log.key_off.push_back(uint32_t(log.key_id.size()));
    log.dep_off.push_back(uint32_t(log.dep_dot.size()));
  }

  // dot + command + deps (Add and RequestReply::Info)
  void add_like(uint8_t kind) {
    const uint64_t d = r.dot();
    uint64_t client, seq, mask;
    uint8_t ro;
    command(client, seq, mask, ro);
    const uint64_t ndeps = r.len();
    for (uint64_t i = 0; i < ndeps; i++) dependency();
    close_event(kind, d, client, seq, mask, ro);
  }

  void dots_event(uint8_t kind, uint64_t from) {
    const uint64_t n = r.len();
    for (uint64_t i = 0; i < n; i++) {
      log.dep_dot.push_back(r.dot());
      log.dep_shards.push_back(0);
    }
    close_event(kind, 0, 0, 0, from, 0);
  }

  void info() {
    switch (r.u32()) {
      case 0: add_like(FH_LOG_ADD); break;
      case 1: dots_event(FH_LOG_REQUEST, r.u64()); break;
      case 2: {
        const uint64_t n = r.len();
        for (uint64_t i = 0; i < n; i++) {
          switch (r.u32()) {
            case 0: add_like(FH_LOG_REPLY_INFO); break;
            case 1: close_event(FH_LOG_REPLY_EXECUTED, r.dot(), 0, 0, 0, 0); break;
            default: r.fail("invalid RequestReply variant");
          }
        }
        break;
      }
      case 3: dots_event(FH_LOG_EXECUTED, 0); break;
      default: r.fail("invalid GraphExecutionInfo variant");
    }
    if (r.p != r.end) r.fail("trailing bytes in frame");
  }
};

}  // namespace

void parse_execlog(ExecLog &log, const uint8_t *buf, size_t len) {
  size_t off = 0;
  while (off < len) {
    FH_CHECK(len - off >= 4, FH_EINVAL,
             "execution log: truncated frame header at byte " + std::to_string(off));
    const uint32_t flen = (uint32_t(buf[off]) << 24) | (uint32_t(buf[off + 1]) << 16) |
                          (uint32_t(buf[off + 2]) << 8) | uint32_t(buf[off + 3]);
    off += 4;
    FH_CHECK(flen <= len - off, FH_EINVAL,
             "execution log: frame " + std::to_string(log.frames) + " longer than the log");
    Parser ps{log, Reader{buf + off, buf + off + flen, log.frames, buf}};
    ps.info();
    off += flen;
    log.frames++;
  }
}

}  // namespace fh

struct fh_execlog {
  fh::ExecLog log;
};

// the replay lives in graph_api.hip (it drives fh_graph); declared there
extern "C" {

fh_status fh_execlog_parse(const uint8_t *buf, size_t len, uint64_t shard_id, fh_execlog **out) {
  FH_API_BEGIN
  FH_CHECK(out && (len == 0 || buf), FH_EINVAL, "null argument");
  auto *h = new fh_execlog();
  h->log.shard_id = shard_id;
  try {
    fh::parse_execlog(h->log, buf, len);
  } catch (...) {
    delete h;
    throw;
  }
  *out = h;
  FH_API_END
}

fh_status fh_execlog_destroy(fh_execlog *h) {
  FH_API_BEGIN
  delete h;
  FH_API_END
}

fh_status fh_execlog_sizes(const fh_execlog *h, size_t *frames, size_t *events, size_t *keys,
                           size_t *deps, size_t *distinct_keys) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  if (frames) *frames = h->log.frames;
  if (events) *events = h->log.kind.size();
  if (keys) *keys = h->log.key_id.size();
  if (deps) *deps = h->log.dep_dot.size();
  if (distinct_keys) *distinct_keys = h->log.key_names.size();
  FH_API_END
}

fh_status fh_execlog_events(const fh_execlog *h, uint8_t *kind, uint64_t *dot,
                            uint64_t *rifl_client, uint64_t *rifl_seq, uint64_t *shards,
                            uint8_t *read_only, uint32_t *key_off, uint64_t *key_id,
                            uint32_t *dep_off, uint64_t *dep_dot, uint64_t *dep_shards) {
  FH_API_BEGIN
  FH_CHECK(h, FH_EINVAL, "null handle");
  const auto &L = h->log;
  auto put = [](auto *dst, const auto &src) {
    if (dst && !src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(src[0]));
  };
  put(kind, L.kind);
  put(dot, L.dot);
  put(rifl_client, L.rifl_client);
  put(rifl_seq, L.rifl_seq);
  put(shards, L.shards);
  put(read_only, L.read_only);
  put(key_off, L.key_off);
  put(key_id, L.key_id);
  put(dep_off, L.dep_off);
  put(dep_dot, L.dep_dot);
  put(dep_shards, L.dep_shards);
  FH_API_END
}

fh_status fh_execlog_key(const fh_execlog *h, uint64_t id, char *buf, size_t cap, size_t *len) {
  FH_API_BEGIN
  FH_CHECK(h && len, FH_EINVAL, "null argument");
  FH_CHECK(id < h->log.key_names.size(), FH_EINVAL, "key id out of range");
  const std::string &k = h->log.key_names[id];
  *len = k.size();
  FH_CHECK(buf && cap >= k.size(), FH_ECAP, "key buffer too small");
  std::memcpy(buf, k.data(), k.size());
  FH_API_END
}

}  // extern "C"

namespace fh {
const ExecLog &execlog_of(const fh_execlog *h) { return h->log; }
}  // namespace fh
