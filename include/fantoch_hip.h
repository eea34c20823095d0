/*
 * fantoch_hip.h -- C ABI of the MI355X batched dependency engine.
 *
 * This is the drop-in boundary for fantoch's dependency hot path: every entry
 * point below replaces one reference interface (cited file:line, paths
 * relative to the reference repository root).  The reference-side binding a
 * maintainer would add (a `fantoch_hip` Rust crate: extern "C" decls,
 * `impl KeyDeps for HipKeyDeps`, `impl Executor for HipGraphExecutor`) is
 * given in INTEGRATION.md.
 *
 * Conventions
 *  - Dots are packed u64: ProcessId (u8) in bits 56..63, sequence in bits
 *    0..55.  The packed order equals the derived Ord of fantoch's
 *    Id{source, sequence} (fantoch/src/id.rs:21-27).  A dot is never 0.
 *  - Keys are dense interned ids `< fh_config.key_space` (fantoch keys are
 *    Strings, fantoch/src/kvs.rs:6; the shim interns them, no hashing, so
 *    there are no collisions).
 *  - All pointers passed in are HOST pointers owned by the caller unless the
 *    name says `_device`; no pointer is retained after a call returns.  The
 *    library owns device state behind opaque handles.
 *  - Every function returns an fh_status.  On error fh_last_error() gives a
 *    thread-local message.  The reference panics on every invariant
 *    violation on this path; the shim turns non-OK into panic!.
 *  - A handle is single-threaded (external synchronisation) and owns one HIP
 *    stream on one device.
 */
#ifndef FANTOCH_HIP_H
#define FANTOCH_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FH_ABI_VERSION 1

typedef enum fh_status {
  FH_OK = 0,
  FH_EINVAL = 1,      /* bad argument (null pointer, key id >= key_space, ...) */
  FH_EHIP = 2,        /* HIP runtime error (no device, launch failure, ...)    */
  FH_EOOM = 3,        /* device allocation failed                              */
  FH_EINVARIANT = 4,  /* internal invariant violated (reference: panic!)       */
  FH_ECAP = 5,        /* output buffer too small; *len receives the size needed,
                         no state was changed                                  */
  FH_ENOTIMPL = 6     /* configuration not supported by this build             */
} fh_status;

/* Mirrors the parts of fantoch::config::Config the hot path reads
 * (fantoch/src/config.rs:7-43) plus device placement. */
typedef struct fh_config {
  uint32_t n;           /* processes per shard            Config::n           */
  uint32_t f;           /* tolerated faults               Config::f           */
  uint32_t shard_count; /* shards                         Config::shard_count */
  int32_t device;       /* HIP device ordinal; -1 = env FANTOCH_HIP_DEVICE,
                           else shard_id % device count          */
  uint64_t key_space;   /* interned key ids are < key_space (<= 2^31)         */
} fh_config;

const char *fh_version(void);
/* Thread-local message for the last non-OK status returned on this thread. */
const char *fh_last_error(void);
fh_status fh_device_count(int *out);

/* ======================================================================
 * KeyDeps -- conflict detection.
 * Replaces SequentialKeyDeps
 * (fantoch_ps/src/protocol/common/graph/deps/keys/sequential.rs:7-144)
 * behind the KeyDeps trait (fantoch_ps/src/protocol/common/graph/deps/keys/
 * mod.rs:37-63).
 * ==================================================================== */
typedef struct fh_keydeps fh_keydeps;

/* KeyDeps::new(shard_id)  keys/mod.rs:39 */
fh_status fh_keydeps_create(uint64_t shard_id, const fh_config *cfg,
                            fh_keydeps **out);
fh_status fh_keydeps_destroy(fh_keydeps *h);

/* A batch of KeyDeps::add_cmd / add_noop calls in arrival order
 * (keys/mod.rs:44-52; sequential.rs:24-42, do_add_cmd :72-104,
 * do_add_noop :106-123).  Result i equals what the i-th sequential call
 * would have returned.
 *   dot[n]                 command dots
 *   key_off[n+1], key_id[] the command's keys on this shard (Command::keys,
 *                          fantoch/src/command.rs:95-100); ignored for noops
 *   is_noop[n]             NULL = no noops
 *   past_off[n+1], past_dot[]  the `past: Option<HashSet<Dependency>>`
 *                          argument (NULL = None for every command)
 *   out_dep_off[n+1], out_dep_dot[out_cap]  dependency dots per command,
 *                          ascending, no duplicates (a HashSet<Dependency>;
 *                          `shards` is a function of the dot)
 * Upper bound needed for out_cap: sum_i(keys_i + past_i + 1) for commands
 * plus (distinct keys seen + 1) per noop; if out_cap is smaller, FH_ECAP is
 * returned with *out_len = that bound and no state changes. */
fh_status fh_keydeps_add_batch(fh_keydeps *h, size_t n, const uint64_t *dot,
                               const uint32_t *key_off, const uint64_t *key_id,
                               const uint8_t *is_noop, const uint32_t *past_off,
                               const uint64_t *past_dot, uint32_t *out_dep_off,
                               uint64_t *out_dep_dot, size_t out_cap,
                               size_t *out_len);

/* fh_keydeps_add_batch with LockedKeyDeps' read/write rules
 * (deps/keys/locked.rs:83-128): per key, a read-only command
 * (read_only[i] = Command::read_only, fantoch/src/command.rs:65-67) depends
 * on the latest write and becomes the latest read; a write depends on the
 * latest read and the latest write and becomes the latest write.  Noops
 * (:130-169) depend on every key's latest read and write.  Write-only
 * batches give SequentialKeyDeps' results.  Upper bound for out_cap:
 * sum_i(2 keys_i + past_i + 1) for commands, plus (2 distinct keys seen + 1)
 * per noop. */
fh_status fh_keydeps_add_batch_rw(fh_keydeps *h, size_t n, const uint64_t *dot,
                                  const uint32_t *key_off, const uint64_t *key_id,
                                  const uint8_t *read_only, const uint8_t *is_noop,
                                  const uint32_t *past_off, const uint64_t *past_dot,
                                  uint32_t *out_dep_off, uint64_t *out_dep_dot,
                                  size_t out_cap, size_t *out_len);

/* fh_keydeps_add_batch on device-resident buffers (the multi-GPU partial-
 * replication path): commands only (no noops, no past), every
 * pointer a device pointer on the handle's device.  key_off_dev[n+1] with
 * key_off_dev[n] == nkeys (given on the host).  The call waits for `stream`
 * (hipStream_t of the caller that produced the inputs, NULL = null stream),
 * runs on the handle's stream and returns when out_off_dev[n+1] and
 * out_dep_dev[*out_len] are written.  out_cap >= nkeys + n, else FH_ECAP with
 * *out_len = that bound and no state change.  FH_EINVAL (after the batch ran)
 * for a key id >= key_space. */
fh_status fh_keydeps_add_batch_device(fh_keydeps *h, size_t n, size_t nkeys,
                                      const uint64_t *dot_dev,
                                      const uint32_t *key_off_dev,
                                      const uint64_t *key_id_dev,
                                      uint32_t *out_off_dev, uint64_t *out_dep_dev,
                                      size_t out_cap, size_t *out_len,
                                      void *stream);

/* KeyDeps::cmd_deps (test-only query, keys/mod.rs:54-56;
 * sequential.rs:44-50): latest noop + latest dot of each key, no update. */
fh_status fh_keydeps_cmd_deps(fh_keydeps *h, size_t nkeys,
                              const uint64_t *key_id, uint64_t *out,
                              size_t cap, size_t *out_len);
/* KeyDeps::noop_deps (keys/mod.rs:58-60; sequential.rs:52-58). */
fh_status fh_keydeps_noop_deps(fh_keydeps *h, uint64_t *out, size_t cap,
                               size_t *out_len);

/* Partial replication: the owner shard's union of every shard's dependency
 * reports for its commands -- Atlas's MShardCommit union
 * (fantoch_ps/src/protocol/atlas.rs:559-639, union at :580-583; each shard's
 * KeyDeps sees Command::keys(shard), fantoch/src/command.rs:95-100).
 * Device pointers on `stream` (a hipStream_t, NULL = null stream) of
 * `device` (-1 = current):
 *   cmd[nrec] (< n_cmd), dep[nrec]   records, any order, duplicates allowed
 *   out_off[n_cmd+1], out_dep[nrec]  per-command deps, ascending, unique
 * *out_len = number of distinct deps (the call synchronises `stream`). */
fh_status fh_dep_union(int device, size_t n_cmd, size_t nrec, const uint32_t *cmd,
                       const uint64_t *dep, uint32_t *out_off, uint64_t *out_dep,
                       size_t *out_len, void *stream);

/* ======================================================================
 * Graph executor -- SCC + execution order.
 * Replaces GraphExecutor / DependencyGraph / TarjanSCCFinder
 * (fantoch_ps/src/executor/graph/executor.rs:19-197, mod.rs:45-679,
 * tarjan.rs:25-359, index.rs:18-211) behind the Executor trait
 * (fantoch/src/executor/mod.rs:27-88).
 * ==================================================================== */
typedef struct fh_graph fh_graph;

/* Executor::new(process_id, shard_id, config)  executor/mod.rs:39;
 * DependencyGraph::new  graph/mod.rs:83-125 */
fh_status fh_graph_create(uint32_t process_id, uint64_t shard_id,
                          const fh_config *cfg, fh_graph **out);
fh_status fh_graph_destroy(fh_graph *h);

/* A batch of GraphExecutionInfo::Add{dot, cmd, deps} in arrival order
 * (executor.rs:78-86 -> DependencyGraph::handle_add, graph/mod.rs:215-277).
 * Vertices whose dependencies are all executed or present are ordered and
 * become drainable; the rest stay pending (carried to later batches) exactly
 * like the reference's PendingIndex (graph/index.rs:145-211). */
fh_status fh_graph_add_batch(fh_graph *h, size_t n, const uint64_t *dot,
                             const uint32_t *key_off, const uint64_t *key_id,
                             const uint32_t *dep_off, const uint64_t *dep_dot);

/* Drain commands ready to execute, in execution order
 * (DependencyGraph::command_to_execute, graph/mod.rs:133-135): SCCs in
 * topological order of the condensation, members of an SCC in dot order
 * (tarjan.rs:14-15, mod.rs:497-524).  scc_label (may be NULL) receives the
 * minimum dot of the command's SCC. */
fh_status fh_graph_drain(fh_graph *h, uint64_t *exec_dot, uint64_t *scc_label,
                         size_t cap, size_t *len);

/* Executed-clock updates (AEClock::add; graph/mod.rs:199-212, 397-405).
 * set_executed_frontier raises a source's contiguous frontier (FH_EINVAL if
 * it would move backwards), dropping exceptions at or below it and folding
 * the ones right above it, as AEClock::add does. */
fh_status fh_graph_mark_executed(fh_graph *h, size_t n, const uint64_t *dot);
fh_status fh_graph_set_executed_frontier(fh_graph *h, uint32_t source,
                                         uint64_t seq);
/* Current time in ms (SysTime::millis of the caller, fantoch/src/time.rs:3-6):
 * vertices added afterwards are stamped with it (Vertex::new,
 * graph/tarjan.rs:335-351) and the execution delay of a command is the time
 * at which it becomes ready minus its stamp (graph/mod.rs:515-520). */
fh_status fh_graph_set_time(fh_graph *h, uint64_t now_ms);
/* Executor::monitor_pending -> VertexIndex::monitor_pending
 * (graph/index.rs:53-103, graph/mod.rs:181-196): the pending vertices
 * pending for >= threshold_ms (the reference uses 1 s), longest first, with
 * the number of missing dependencies found through other pending vertices
 * (missing_dependencies, index.rs:105-142).  FH_EINVARIANT if one of them
 * has none (the reference panics: a liveness bug).  Any array may be NULL;
 * *len = count (up to cap entries written). */
fh_status fh_graph_monitor_pending(fh_graph *h, uint64_t threshold_ms,
                                   uint64_t *dots, uint64_t *pending_ms,
                                   uint64_t *missing, size_t cap, size_t *len);
/* Executor metrics collected since the last call (ExecutorMetricsKind,
 * fantoch/src/executor/mod.rs:120-129, collected in save_scc,
 * graph/mod.rs:490-525): chain_size[] = the size of every executed SCC
 * (ChainSize), exec_delay[] = ms from add to ready of every executed command
 * (ExecutionDelay).  FH_ECAP (counts set, nothing taken) if a cap is short. */
fh_status fh_graph_take_metrics(fh_graph *h, uint64_t *chain_size, size_t chain_cap,
                                uint64_t *exec_delay, size_t delay_cap,
                                size_t *n_chain, size_t *n_delay);
/* Graph passes run and pending retries skipped (a retry with no new vertex
 * where none of the pending set's missing dependencies executed since the
 * last pass), for tests and tuning. */
fh_status fh_graph_passes(fh_graph *h, uint64_t *passes, uint64_t *skipped);
/* Number of pending vertices (VertexIndex size, graph/index.rs:18-51). */
fh_status fh_graph_pending(fh_graph *h, size_t *count);
/* Missing dependencies of pending vertices (deps neither executed nor
 * indexed; the dots PendingIndex waits on, index.rs:171-205). */
fh_status fh_graph_missing(fh_graph *h, uint64_t *dots, size_t cap,
                           size_t *len);
/* Fault injection and a self-test of the small pass's completion wait
 * (tests only; no reference counterpart: the reference's executor cannot
 * hang on a device).  fh_graph_inject_small_delay makes every later small
 * pass (graph_small.hip) wait delay_us on the device before it starts, and
 * sets the host's completion deadline to deadline_ms (0 keeps the default,
 * 30,000): a pass that misses it returns FH_EHIP with fh_last_error() set,
 * and the handle then refuses every call but fh_graph_destroy (which waits
 * for the kernel).  fh_selftest_poll_deadline runs the same host wait
 * against a stream that never completes (no GPU needed) and returns the
 * status it raised: FH_EHIP. */
fh_status fh_graph_inject_small_delay(fh_graph *h, uint32_t delay_us, uint32_t deadline_ms);
fh_status fh_selftest_poll_deadline(uint32_t deadline_ms);

/* ---- Partial replication: requests and replies between shards ----------
 * (graph/mod.rs:139-157, 168-179, 279-408; index.rs:145-211;
 * GraphExecutor::{cleanup, fetch_requests, fetch_request_replies,
 * handle(Request/RequestReply)} executor.rs:65-70, 147-189, 242-262).
 * One fh_graph plays both executor roles of a shard (index 0 adds, index 1
 * answers requests); they share the vertex index in the reference too
 * (index.rs:21), and the executed clock the replies consult is the main
 * executor's (the reference's secondary clock is that clock, delivered by
 * handle_executed). */

/* fh_graph_add_batch with shard sets, as 64-bit masks (bit s = shard s):
 * cmd_shards[n] = Command::shards() of each added command (command.rs:103-
 * 110), dep_shards[dep_off[n]] = Dependency::shards of each dependency
 * (deps/keys/mod.rs:18-35).  A dependency missing when its command is added
 * whose shard set excludes this shard is queued as a request to
 * Dot::target_shard(n) (id.rs:59-61) the first time it is indexed
 * (PendingIndex::index, index.rs:171-205).  FH_EINVARIANT for a missing
 * dependency with an empty shard set (a noop: index.rs:190-194). */
fh_status fh_graph_add_batch_sharded(fh_graph *h, size_t n, const uint64_t *dot,
                                     const uint32_t *key_off, const uint64_t *key_id,
                                     const uint32_t *dep_off, const uint64_t *dep_dot,
                                     const uint64_t *cmd_shards,
                                     const uint64_t *dep_shards);
/* DependencyGraph::requests (mod.rs:147-150): take the queued requests,
 * sorted by (target shard, dot).  FH_ECAP (len = count, nothing taken) if
 * cap is too small. */
fh_status fh_graph_requests(fh_graph *h, uint64_t *dot, uint64_t *shard,
                            size_t cap, size_t *len);
/* handle_request / process_requests (mod.rs:279-375): per dot, an Info
 * reply {dot, deps, shard sets} for a pending vertex (FH_EINVARIANT if the
 * vertex's command is replicated by from_shard, :313-322), an Executed reply
 * for an executed dot, otherwise buffered until fh_graph_cleanup. */
fh_status fh_graph_handle_requests(fh_graph *h, uint64_t from_shard, size_t n,
                                   const uint64_t *dots);
/* cleanup -> check_pending_requests (mod.rs:168-179, 673-678). */
fh_status fh_graph_cleanup(fh_graph *h);
#define FH_REPLY_INFO 0     /* RequestReply::Info{dot, cmd, deps}  mod.rs:33-43 */
#define FH_REPLY_EXECUTED 1 /* RequestReply::Executed{dot}                      */
/* DependencyGraph::request_replies (mod.rs:152-157): take the queued
 * replies.  Reply i goes to to_shard[i]; Info replies carry the vertex's
 * deps in dep_dot/dep_shards[dep_off[i]..dep_off[i+1]] (the command payload
 * stays with the caller, keyed by dot).  FH_ECAP (counts set, nothing taken)
 * if cap < replies or dep_cap < deps.  The receiver applies Info with
 * fh_graph_add_batch_sharded and Executed with fh_graph_mark_executed
 * followed by an empty add batch (the pending retry, mod.rs:393-405). */
fh_status fh_graph_request_replies(fh_graph *h, size_t cap, uint64_t *to_shard,
                                   uint8_t *kind, uint64_t *dot,
                                   uint64_t *cmd_shards, uint32_t *dep_off,
                                   size_t dep_cap, uint64_t *dep_dot,
                                   uint64_t *dep_shards, size_t *n_replies,
                                   size_t *n_deps);

/* ---- Execution-log ingest and replay ---------------
 * The runner's execution log (run/task/execution_logger.rs:11-55): frames of
 * a 4-byte big-endian length (tokio LengthDelimitedCodec defaults,
 * run/rw/mod.rs:20-36) holding a bincode-1.3 GraphExecutionInfo
 * (executor/graph/executor.rs:204-222; run/rw/mod.rs:87-100).  Replaces the
 * replay binary's loop (fantoch_ps/src/bin/graph_executor_replay.rs:13-38).
 * Host-only parsing: no device is needed to parse. */
typedef struct fh_execlog fh_execlog;
#define FH_LOG_ADD 0            /* GraphExecutionInfo::Add{dot, cmd, deps}  */
#define FH_LOG_REQUEST 1        /* ::Request{from, dots}                    */
#define FH_LOG_REPLY_INFO 2     /* ::RequestReply -> RequestReply::Info     */
#define FH_LOG_REPLY_EXECUTED 3 /* ::RequestReply -> RequestReply::Executed */
#define FH_LOG_EXECUTED 4       /* ::Executed{dots}                         */
/* Parse a whole log; Command::keys(shard_id) become each event's keys
 * (interned in first-seen order).  FH_EINVAL names the frame and byte of
 * malformed input (bad variant / tag, truncation, trailing bytes). */
fh_status fh_execlog_parse(const uint8_t *buf, size_t len, uint64_t shard_id,
                           fh_execlog **out);
fh_status fh_execlog_destroy(fh_execlog *h);
/* Sizes for fh_execlog_events: frames, events, keys (sum over events),
 * deps (sum over events), distinct keys.  Any pointer may be NULL. */
fh_status fh_execlog_sizes(const fh_execlog *h, size_t *frames, size_t *events,
                           size_t *keys, size_t *deps, size_t *distinct_keys);
/* Event arrays (any pointer may be NULL): kind[events], dot[events] (packed),
 * rifl_client/rifl_seq[events], shards[events] (Command::shards() mask, or
 * the requesting shard of a Request), read_only[events],
 * key_off[events+1] / key_id[keys], dep_off[events+1] / dep_dot[deps] /
 * dep_shards[deps] (Dependency::shards mask, 0 = None; the dots of a
 * Request / Executed). */
fh_status fh_execlog_events(const fh_execlog *h, uint8_t *kind, uint64_t *dot,
                            uint64_t *rifl_client, uint64_t *rifl_seq,
                            uint64_t *shards, uint8_t *read_only,
                            uint32_t *key_off, uint64_t *key_id,
                            uint32_t *dep_off, uint64_t *dep_dot,
                            uint64_t *dep_shards);
/* Name of interned key `id` (FH_ECAP with *len = size if cap is short). */
fh_status fh_execlog_key(const fh_execlog *h, uint64_t id, char *buf,
                         size_t cap, size_t *len);
/* Feed the log to an executor as GraphExecutor::handle would
 * (executor.rs:76-100): runs of Add / RequestReply::Info events go in
 * batches of up to `batch` (0 = unbounded) to fh_graph_add_batch_sharded,
 * Request -> fh_graph_handle_requests, RequestReply::Executed ->
 * fh_graph_mark_executed + pending retry, Executed -> nothing (one handle
 * holds the clock).  *executed (may be NULL) = commands that became ready;
 * drain them with fh_graph_drain. */
fh_status fh_execlog_replay(const fh_execlog *h, fh_graph *g, size_t batch,
                            size_t *executed);

/* ======================================================================
 * Caesar's predecessors executor.
 * Replaces PredecessorsExecutor / PredecessorsGraph
 * (fantoch_ps/src/executor/pred/executor.rs, mod.rs:26-352) behind the
 * Executor trait (fantoch/src/executor/mod.rs:27-88); Caesar wires it as its
 * executor (fantoch_ps/src/protocol/caesar.rs:49).
 * ==================================================================== */
typedef struct fh_pred fh_pred;

/* PredecessorsGraph::new(process_id, config) (mod.rs:42-67). */
fh_status fh_pred_create(uint32_t process_id, uint64_t shard_id,
                         const fh_config *cfg, fh_pred **out);
fh_status fh_pred_destroy(fh_pred *h);
/* A batch of PredecessorsGraph::add(dot, cmd, clock, deps) calls in arrival
 * order (mod.rs:89-130).  clock[i] = (Clock.seq << 8) | Clock.process_id
 * (integer order == Clock's Ord, protocol/common/pred/clocks/mod.rs:15-30).
 * A command runs once every dep is committed and every dep with a lower
 * clock has run; ready commands drain in clock order.  FH_EINVARIANT (no
 * state change) for a dot already added (mod.rs:264-273). */
fh_status fh_pred_add_batch(fh_pred *h, size_t n, const uint64_t *dot,
                            const uint64_t *clock, const uint32_t *dep_off,
                            const uint64_t *dep_dot);
/* command_to_execute (mod.rs:71-73), up to cap dots. */
fh_status fh_pred_drain(fh_pred *h, uint64_t *exec_dot, size_t cap,
                        size_t *len);
/* commands still waiting (phase one or two). */
fh_status fh_pred_pending(fh_pred *h, size_t *count);

/* ======================================================================
 * Caesar's KeyClocks -- the timestamp-ordered conflict index whose
 * predecessors become a command's dependencies.
 * Replaces SequentialKeyClocks
 * (fantoch_ps/src/protocol/common/pred/clocks/keys/sequential.rs:14-152)
 * behind the KeyClocks trait (pred/clocks/keys/mod.rs:13-45).  Clocks are
 * packed (seq << 8) | process_id: the integer order is Clock's derived Ord
 * (pred/clocks/mod.rs:15-30).  Dependency sets come back in ascending clock
 * order, without repeats.
 * ==================================================================== */
typedef struct fh_keyclocks fh_keyclocks;
/* KeyClocks::new(process_id, shard_id) (sequential.rs:22-30). */
fh_status fh_keyclocks_create(uint32_t process_id, uint64_t shard_id,
                              const fh_config *cfg, fh_keyclocks **out);
fh_status fh_keyclocks_destroy(fh_keyclocks *h);
/* clock_next / clock_join (sequential.rs:33-42). */
fh_status fh_keyclocks_clock_next(fh_keyclocks *h, uint64_t *clock);
fh_status fh_keyclocks_clock_join(fh_keyclocks *h, uint64_t clock);
/* A batch of KeyClocks::add(dot, cmd, clock) (sequential.rs:43-56): each
 * command's keys (key_off[n+1], key_id[]) get the entry clock -> dot.
 * FH_EINVARIANT (no state change) for a timestamp added twice on a key.
 * Commands of more than 8 keys: FH_ENOTIMPL (the reference takes any
 * number; the device merge holds 8 key segments), here and in remove /
 * predecessors. */
fh_status fh_keyclocks_add(fh_keyclocks *h, size_t n, const uint64_t *dot,
                           const uint32_t *key_off, const uint64_t *key_id,
                           const uint64_t *clock);
/* A batch of KeyClocks::remove(cmd, clock) (sequential.rs:58-75).
 * FH_EINVARIANT (no state change) for a timestamp never added. */
fh_status fh_keyclocks_remove(fh_keyclocks *h, size_t n, const uint32_t *key_off,
                              const uint64_t *key_id, const uint64_t *clock);
/* A batch of KeyClocks::predecessors(dot, cmd, clock, higher)
 * (sequential.rs:77-119): pred_off[n+1] / pred_dot[] = the dots on the
 * command's keys with a lower clock; higher_off / higher_dot (all three
 * higher_* NULL = `higher: None`) = those with a higher clock, each row in
 * ascending (clock, dot) order, one entry per distinct dot (the reference's
 * HashSet<Dot>: two dots holding one clock on different keys are both
 * reported; the same dot on several keys once).  Sizes are
 * always reported (*pred_len, *higher_len); FH_ECAP if a cap is short
 * (nothing written there).  FH_EINVARIANT if another command holds the same
 * timestamp on a key (:108-112). */
fh_status fh_keyclocks_predecessors(fh_keyclocks *h, size_t n, const uint64_t *dot,
                                    const uint32_t *key_off, const uint64_t *key_id,
                                    const uint64_t *clock, uint32_t *pred_off,
                                    uint64_t *pred_dot, size_t pred_cap,
                                    size_t *pred_len, uint32_t *higher_off,
                                    uint64_t *higher_dot, size_t higher_cap,
                                    size_t *higher_len);
/* Entries held (sum over keys of CommandsPerKey sizes). */
fh_status fh_keyclocks_len(fh_keyclocks *h, size_t *entries);

/* ======================================================================
 * Fused engine -- a committed command stream, device resident end to end:
 * KeyDeps (one replica, or the fast-quorum views of Atlas/EPaxos with the
 * QuorumDeps union, quorum.rs:28-98) -> dependency graph -> SCC ->
 * execution order -> per-key execution sequence (ExecutionOrderMonitor,
 * fantoch/src/executor/monitor.rs:20-28).  This is the batched entry the
 * throughput metric is measured on.
 * ==================================================================== */
typedef struct fh_engine fh_engine;

typedef struct fh_stream_desc {
  size_t n;               /* commands in the batch                         */
  uint32_t keys_per_cmd;  /* k: fixed keys per command (<= 8)              */
  uint32_t views;         /* 0 = single replica view (stream order);
                             >0 = fast-quorum size fq (replica views)      */
  uint32_t nproc;         /* processes (replica ids 1..nproc) when views>0 */
  uint32_t flags;         /* FH_STREAM_ELEMENT_LOGS: fh_engine_stage_logs'
                             entries are element positions               */
} fh_stream_desc;
/* fh_engine_stage_logs: log entries are elements, not commands -- position
 * (c*views + j)*k + s = key slot s of command c as fast-quorum member j of
 * that slot's collect.  This is how partial replication stages (each shard's
 * replicas see only the command's keys on their shard, Command::keys(shard),
 * command.rs:95-100); every position of a batch appears in exactly one log,
 * and nproc may reach 64. */
#define FH_STREAM_ELEMENT_LOGS 1u

fh_status fh_engine_create(const fh_config *cfg, fh_engine **out);
fh_status fh_engine_destroy(fh_engine *h);
/* Reset all persistent state (latest tables, executed clock). */
fh_status fh_engine_reset(fh_engine *h);
/* Stage a batch into device memory (host -> HBM, not part of the timed
 * path).  Dots must have a ProcessId >= 1 and must not be the all-ones dot
 * (255, 2^56 - 1), reserved by the union (FH_EINVAL).
 * key_id[n*k]; for views>0, fq_proc[n*fq] (replica of each member,
 * member 0 = coordinator) and fq_time[n*fq] (arrival time of the command at
 * that member; members process commands in (time, index) order). */
fh_status fh_engine_stage(fh_engine *h, const fh_stream_desc *desc,
                          const uint64_t *dot, const uint64_t *key_id,
                          const uint8_t *fq_proc, const uint64_t *fq_time);
/* Stage `nbatches` consecutive batches of desc->n commands each (arrays hold
 * nbatches * n commands, batch-major).  Each fh_engine_run processes the next
 * staged batch, carrying KeyDeps and executed-clock state from the previous
 * one (a committed stream fed batch by batch). */
fh_status fh_engine_stage_many(fh_engine *h, const fh_stream_desc *desc,
                               size_t nbatches, const uint64_t *dot,
                               const uint64_t *key_id, const uint8_t *fq_proc,
                               const uint64_t *fq_time);
/* Stage replica views as the replicas' own arrival logs (views >= 1): the
 * commands replica r + 1's KeyDeps processes, in the order it processes them
 * (its add_cmd calls: coordinator, atlas.rs:236 / epaxos.rs:208, and fast-
 * quorum member, atlas.rs:303-309 / epaxos.rs:275-281).  For batch b and
 * replica r (0 <= r < nproc) the log is log_cmd[log_off[b*nproc + r] ..
 * log_off[b*nproc + r + 1]), batch-local command indices; every command of a
 * batch appears in exactly `views` logs, at most once per log
 * (log_off[nbatches*nproc] == nbatches * n * views).  fh_engine_stage with
 * fq_proc / fq_time builds these logs on the host (members process commands
 * in (time, index) order). */
fh_status fh_engine_stage_logs(fh_engine *h, const fh_stream_desc *desc,
                               size_t nbatches, const uint64_t *dot,
                               const uint64_t *key_id, const uint64_t *log_off,
                               const uint32_t *log_cmd);
/* Replay the staged batches from a clean state (latest tables and executed
 * clock cleared on the engine's stream, no host synchronisation; the next
 * run processes the first staged batch again). */
fh_status fh_engine_rewind(fh_engine *h);
/* Block until every run issued on the engine's stream has finished (what a
 * timed loop of fh_engine_run(h, NULL) calls brackets itself with: the
 * library's HIP runtime is not the caller's, so a device-wide synchronise
 * of another runtime, e.g. torch's, does not wait for it). */
fh_status fh_engine_sync(fh_engine *h);
/* Run the next staged batch on the device (inputs already resident).  If
 * device_ms is non-NULL the stream is synchronised and the device time of
 * the run (HIP events on the engine's stream) is returned. */
fh_status fh_engine_run(fh_engine *h, float *device_ms);
/* Copy the last run's results back; run() materialises them on the device
 * (each pointer may be NULL):
 *   dep_off[n+1], dep_dot[cap]   committed deps per command (ascending)
 *   scc_label[n]                 min dot of each command's SCC
 *   exec_rank[n]                 position of each command in exec order
 *   key_off[key_space+1], key_seq[n*k]  per-key execution sequence (dots) */
fh_status fh_engine_results(fh_engine *h, uint32_t *dep_off, uint64_t *dep_dot,
                            size_t dep_cap, size_t *dep_len,
                            uint64_t *scc_label, uint32_t *exec_rank,
                            uint32_t *key_off, uint64_t *key_seq);
/* Per-kernel device times of the last run (ms), for the roofline report.
 * names/ms arrays of length cap; *len = number of recorded kernels. */
fh_status fh_engine_kernel_times(fh_engine *h, const char **names, float *ms,
                                 size_t cap, size_t *len);
/* Roofline probe: record HIP events (on the engine's stream) around every
 * launch of the named kernels during subsequent runs (comma-separated:
 * "kb_partition", "kb_order" = the two single-view launches, "sort_scatter"
 * = the key+value radix passes, "sv_deps", "sv_tails"; NULL = off), then
 * report a kernel's average device duration and the algorithmic bytes one
 * launch moves (probe_stats: the first named kernel). */
fh_status fh_engine_set_probe(fh_engine *h, const char *kernel);
fh_status fh_engine_probe_stats(fh_engine *h, float *avg_ms, size_t *launches,
                                double *bytes_per_launch);
fh_status fh_engine_probe_stats_for(fh_engine *h, const char *kernel, float *avg_ms,
                                    size_t *launches, double *bytes_per_launch);
/* Enable/disable per-kernel event timing (adds events between kernels). */
fh_status fh_engine_set_profiling(fh_engine *h, int on);
/* Deps-only runs (on != 0): run() stops after the committed deps (KeyDeps
 * per replica view + the QuorumDeps union, quorum.rs:28-98) -- the
 * per-shard stage of partial replication, whose graph runs after the
 * cross-shard union (MShardCommit, atlas.rs:559-639).  results() then
 * returns the deps only (FH_EINVAL for labels, ranks or per-key output). */
fh_status fh_engine_set_deps_only(fh_engine *h, int on);
/* Forget what earlier runs taught the graph stage: the tile kernel's first
 * reach bound (the last run's maximum excess, plus a margin) and the global
 * path's entry (straight to the full coloring when the last run needed it).
 * The next run starts from the defaults, as on a fresh engine; results are
 * the same either way (every run re-checks its certificate).  For cold-run
 * measurements. */
fh_status fh_engine_forget_tuning(fh_engine *h);

/* ======================================================================
 * Multi-GPU fused engine from one process: one engine
 * per device over key shards, owner(key) from fh_key_owners_balanced over
 * the staged stream's key counts.  With one key per
 * command a shard's dependency graph is closed (every dependency joins two
 * commands of one key), so shards order concurrently with no exchange; each
 * keeps the global dots and its replicas' logs restricted to its commands.
 * (Multi-key cross-shard streams go through fh_dep_union and the partial-
 * replication executor instead: FH_ENOTIMPL for keys_per_cmd > 1.)
 * ==================================================================== */
typedef struct fh_multi fh_multi;
/* devices[ndev] (NULL = 0..ndev-1; a device may repeat). */
fh_status fh_multi_create(const fh_config *cfg, size_t ndev,
                          const int32_t *devices, fh_multi **out);
fh_status fh_multi_destroy(fh_multi *h);
/* One batch in the fh_engine_stage_logs layout (global command indices). */
fh_status fh_multi_stage_logs(fh_multi *h, const fh_stream_desc *desc,
                              const uint64_t *dot, const uint64_t *key_id,
                              const uint64_t *log_off, const uint32_t *log_cmd);
fh_status fh_multi_rewind(fh_multi *h);
/* fh_engine_sync on every shard. */
fh_status fh_multi_sync(fh_multi *h);
/* Every shard on its device concurrently (a host thread per device);
 * device_ms (may be NULL) = the slowest shard's device time. */
fh_status fh_multi_run(fh_multi *h, float *device_ms);
/* Merged in the stream's command order (as fh_engine_results): deps, SCC
 * labels, exec_rank = the shards' execution orders concatenated (shards
 * share no dependency), per-key sequences from each key's owner. */
fh_status fh_multi_results(fh_multi *h, uint32_t *dep_off, uint64_t *dep_dot,
                           size_t dep_cap, size_t *dep_len, uint64_t *scc_label,
                           uint32_t *exec_rank, uint32_t *key_off,
                           uint64_t *key_seq);
/* Commands staged on shard `shard`. */
fh_status fh_multi_shard_size(fh_multi *h, size_t shard, size_t *n);
/* The key -> shard map of the last staging (owner[key_space]). */
fh_status fh_multi_owners(fh_multi *h, uint32_t *owner);
/* A balanced key -> shard map from per-key command counts (hist[key_space]):
 * keys in decreasing count (ties: ascending key) each go to the least loaded
 * shard so far (ties: the lowest shard) -- greedy longest-processing-time
 * packing, so a Zipf-hot key fills a shard and the tail evens the rest
 * (max shard <= mean + the largest count).  Deterministic: every rank that
 * passes the same counts gets the same map.  Replaces key % nshards, which
 * under Zipf 0.99 over 2^20 keys puts 1.37x the mean on the largest of 8
 * shards (the reference assigns key shards by hash,
 * fantoch/src/client/workload.rs:203-205). */
fh_status fh_key_owners_balanced(const uint64_t *hist, size_t key_space, uint32_t nshards,
                                 uint32_t *owner);

/* ======================================================================
 * Partial replication across GPUs (BASELINE config C5): one
 * process per GPU, rank q of N; the exchanges between the steps are the
 * caller's (torch.distributed / RCCL over xGMI), every buffer argument named
 * _dev is a device pointer on the handle's device, and every call returns
 * with the handle's stream idle.  Replaces, for a whole committed stream,
 * the shards' collects and MShardCommit union (atlas.rs:214-328, 559-639)
 * and the GraphExecutors that reach other shards' vertices through
 * requests and replies (executor/graph/mod.rs:279-408, index.rs:171-205).
 *   1. KeyDeps by key shard: rank q runs the processes of the shards h with
 *      h % N == q (element logs, Command::keys(shard), command.rs:95-100).
 *   2. Union by stream position: rank q owns commands [a_q, a_q+1) (a_q =
 *      n*q/N); each element's dependency code goes to its command's owner
 *      (all-to-all), which unions each command's keys x views.
 *   3. Local SCCs of the range (cross-range edges cut); vertices reaching a
 *      cross-range edge are contracted to their local SCCs.
 *   4. The condensed graph (those super vertices, plus the ready times of
 *      settled vertices they reach): cross-range targets resolved by their
 *      owners (all-to-all of queries and answers), every rank's part
 *      gathered (all-gather) and solved on every rank.
 *   5. Each (key, command) element goes to the key's owner ((key % shards)
 *      % N, all-to-all) with its order key; per-key sequences are sorted
 *      there.
 * Outputs per rank: the committed deps and SCC labels of its range, the
 * per-key execution sequences of its keys (ExecutionOrderMonitor,
 * fantoch/src/executor/monitor.rs:20-28).
 * ==================================================================== */
typedef struct fh_dgraph fh_dgraph;
fh_status fh_dgraph_create(const fh_config *cfg, uint32_t rank, uint32_t world,
                           fh_dgraph **out);
fh_status fh_dgraph_destroy(fh_dgraph *h);
/* The whole stream's dot[n] / key_id[n*k] (host) and this rank's processes'
 * element logs (desc->flags has FH_STREAM_ELEMENT_LOGS, desc->nproc = its
 * logs: the processes of its shards, shard order).  send_counts[world] /
 * recv_counts[world] = elements of the code exchange; range[2] = (a_q,
 * commands in the range). */
fh_status fh_dgraph_stage(fh_dgraph *h, const fh_stream_desc *desc, uint32_t shards,
                          const uint64_t *dot, const uint64_t *key_id,
                          const uint64_t *log_off, const uint32_t *log_elem,
                          uint64_t *send_counts, uint64_t *recv_counts,
                          uint64_t *range);
/* Step 1: this rank's KeyDeps; its elements' codes, by destination. */
fh_status fh_dgraph_keydeps(fh_dgraph *h, uint32_t *send_dev);
/* Steps 2-3: the range's codes (by source) -> union, local SCCs, escaping
 * set; query_counts[world] = cross-range targets to resolve per owner. */
fh_status fh_dgraph_local(fh_dgraph *h, const uint32_t *recv_dev,
                          uint64_t *query_counts);
fh_status fh_dgraph_queries(fh_dgraph *h, uint32_t *query_dev);
/* An owner's answers to n queried vertices of its range. */
fh_status fh_dgraph_answer(fh_dgraph *h, size_t n, const uint32_t *in_dev,
                           uint32_t *out_dev);
/* Step 4: with the answers, this rank's part of the condensed graph: nv
 * vertices (2 x u64 each), ne edges (u64 each). */
fh_status fh_dgraph_condense(fh_dgraph *h, const uint32_t *answers_dev, uint64_t *nv,
                             uint64_t *ne);
fh_status fh_dgraph_condensed_part(fh_dgraph *h, uint64_t *verts_dev, uint64_t *edges_dev);
/* Step 5: every rank's parts (gathered) -> solve, order keys of the range;
 * elem_counts[world] = per-key elements for each key owner. */
fh_status fh_dgraph_solve(fh_dgraph *h, size_t nv, const uint64_t *verts_dev, size_t ne,
                          const uint64_t *edges_dev, uint64_t *elem_counts);
fh_status fh_dgraph_elements(fh_dgraph *h, uint64_t *elem_dev);
/* The n elements of this rank's keys (2 x u64 each) -> per-key sequences. */
fh_status fh_dgraph_per_key(fh_dgraph *h, size_t n, const uint64_t *elem_dev);
/* Host copies (any pointer may be NULL): the range's committed deps
 * (dep_off[count+1], dep_dot), SCC labels (min dot) of the range's commands,
 * and the per-key elements of this rank's keys, by key then execution
 * order (pk_key[*pk_len], pk_dot[*pk_len]). */
fh_status fh_dgraph_results(fh_dgraph *h, uint32_t *dep_off, uint64_t *dep_dot,
                            size_t dep_cap, size_t *dep_len, uint64_t *scc_label,
                            uint32_t *pk_key, uint64_t *pk_dot, size_t *pk_len);
/* Device time of each step of the last run (profiling on). */
fh_status fh_dgraph_set_profiling(fh_dgraph *h, int on);
fh_status fh_dgraph_stage_times(fh_dgraph *h, const char **names, float *ms, size_t cap,
                                size_t *len);

/* ======================================================================
 * Synthetic workload (fantoch/src/client/{workload,key_gen}.rs semantics,
 * seeded and counter-based so every consumer sees the same stream).
 * ==================================================================== */
typedef struct fh_workload {
  uint64_t seed;
  uint32_t n;             /* processes per shard (dot sources 1..n)        */
  uint32_t keys_per_cmd;  /* k                                             */
  uint32_t kind;          /* 0 = Zipf{s, key_count}; 1 = ConflictRate{r};
                             2 = ConflictPool{r, pool} (key0 = shared key
                             with prob r%, key1.. from a pool)             */
  uint32_t conflict_rate; /* percent, kinds 1/2                            */
  uint32_t pool_size;     /* kind 2                                        */
  uint32_t clients;       /* clients (round-robin submission), kinds 1/2   */
  double zipf_s;          /* kind 0                                        */
  uint64_t key_count;     /* kind 0: keys ranked 1..key_count -> ids 0..   */
  uint32_t views;         /* fast quorum size (0 = single view)            */
  uint32_t window;        /* reorder window W for replica views            */
  uint32_t shards;        /* 0 or 1 = full replication; >= 2 = partial
                             replication over `shards` key shards (key %
                             shards), n processes each (n * shards <= 255):
                             shard h = processes n*h+1 .. n*h+n
                             (fantoch/src/util.rs:115-122); a command's dot
                             comes from its first key's shard (its target
                             shard, client/workload.rs:172-176, id.rs:59-61),
                             and every shard it touches collects it with
                             its own fast quorum and arrival delays
                             (atlas.rs:214-328; union atlas.rs:559-639)    */
  uint32_t pad;
} fh_workload;

/* Key space the workload's ids live in. */
uint64_t fh_workload_key_space(const fh_workload *w);
/* Generate commands [first, first+count): dot[count], key_id[count*k] and,
 * if views>0, fq_proc[count*views], fq_time[count*views].  Partial
 * replication (shards >= 2): fq_proc / fq_time are per key slot,
 * [(c*k + s)*views + j] = view j of the collect in key slot s's shard. */
fh_status fh_workload_generate(const fh_workload *w, uint64_t first,
                               size_t count, uint64_t *dot, uint64_t *key_id,
                               uint8_t *fq_proc, uint64_t *fq_time);
/* The same commands' replica views as per-replica arrival logs (the
 * fh_engine_stage_logs layout for one batch): log_off[n+1] (n = processes),
 * log_cmd[count*views] batch-local command indices; replica r lists the
 * commands it is a member for in (fq_time, index) order. */
fh_status fh_workload_generate_logs(const fh_workload *w, uint64_t first,
                                    size_t count, uint64_t *log_off,
                                    uint32_t *log_cmd);
/* The same commands' replica views as element logs (the fh_engine_stage_logs
 * layout with FH_STREAM_ELEMENT_LOGS, one batch): log_off[n*S+1] (S = shards,
 * 1 when unsharded; log r = process r+1), log_elem[count*k*views] element
 * positions (c*views + j)*k + s: process r's KeyDeps sees key slot s of
 * command c as member j of the slot's shard's fast quorum, in (time, c, s)
 * order.  Every element appears in exactly one log. */
fh_status fh_workload_generate_element_logs(const fh_workload *w, uint64_t first,
                                            size_t count, uint64_t *log_off,
                                            uint32_t *log_elem);
/* Key shard `shard` of nshards of commands [first, first+count): the
 * commands whose first key k0 has k0 % nshards == shard (the key's owner,
 * SURVEY §8e), in stream order with their global dots; *n_out = how many.
 * All output pointers NULL = size query.  log_off[n+1] / log_cmd[*n_out *
 * views] (both NULL = no logs): the replicas' arrival logs restricted to the
 * shard, as shard-local command indices. */
fh_status fh_workload_generate_shard(const fh_workload *w, uint64_t first,
                                     size_t count, uint32_t nshards,
                                     uint32_t shard, size_t *n_out,
                                     uint64_t *dot, uint64_t *key_id,
                                     uint64_t *log_off, uint32_t *log_cmd);
/* The same with an explicit key -> shard map (owner[key_space], e.g.
 * fh_key_owners_balanced; NULL = key % nshards): the commands whose first
 * key k0 has owner[k0] == shard. */
fh_status fh_workload_generate_shard_owned(const fh_workload *w, uint64_t first,
                                           size_t count, const uint32_t *owner,
                                           uint32_t nshards, uint32_t shard,
                                           size_t *n_out, uint64_t *dot,
                                           uint64_t *key_id, uint64_t *log_off,
                                           uint32_t *log_cmd);
/* hist[key_space]: how many of commands [first, first+count) have each key
 * as their first key (the input of fh_key_owners_balanced). */
fh_status fh_workload_key_histogram(const fh_workload *w, uint64_t first,
                                    size_t count, uint64_t *hist);

#ifdef __cplusplus
}
#endif
#endif /* FANTOCH_HIP_H */
