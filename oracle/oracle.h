/*
 * oracle.h -- CPU restatement of fantoch's dependency hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / timed CPU baseline.
 *
 * Parity status: pinned.  The reference (Rust, edition 2018) cannot be
 * compiled in this image (no cargo/rustc, crates not vendored -- see
 * DESIGN.md "Oracle").  This restatement is pinned by the reference's own
 * known-answer tests, transcribed as fixtures under tests/golden/:
 *   key_deps_flow       fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:98-329
 *   QuorumDeps tests    fantoch_ps/src/protocol/common/graph/deps/quorum.rs:114-287
 *   simple / cycle / test_add_random / sccs_found_and_missing_dep /
 *   transitive_conflicts_assumption_regression_test_{1,2}
 *                       fantoch_ps/src/executor/graph/mod.rs:716-1350
 *   simple / already_mutably_borrowed_regression_test / test_add_random
 *   (Caesar)            fantoch_ps/src/executor/pred/mod.rs:386-687
 *                       (tests/test_oracle_pred.py)
 *
 * Dots are packed u64: source (ProcessId, u8) in bits 56..63, sequence in
 * bits 0..55.  Packed order == the derived Ord of Id{source, sequence}
 * (fantoch/src/id.rs:21-27).
 */
#ifndef FANTOCH_ORACLE_H
#define FANTOCH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FO_DOT(src, seq) ((((uint64_t)(src)) << 56) | ((uint64_t)(seq)))
#define FO_SRC(d) ((uint32_t)((d) >> 56))
#define FO_SEQ(d) ((d) & 0x00FFFFFFFFFFFFFFULL)

/* ---------------------------------------------------------------------
 * SequentialKeyDeps  (deps/keys/sequential.rs:7-144)
 * ------------------------------------------------------------------- */
typedef struct fo_keydeps fo_keydeps;

fo_keydeps *fo_keydeps_new(uint64_t shard_id);
void fo_keydeps_free(fo_keydeps *kd);
/* add_cmd (sequential.rs:24-36, do_add_cmd :72-104).  `past` may be NULL
 * (None).  Writes the dep set sorted ascending into out (if cap allows) and
 * returns its size. */
size_t fo_keydeps_add_cmd(fo_keydeps *kd, uint64_t dot, const uint64_t *keys,
                          size_t nkeys, const uint64_t *past, size_t npast,
                          int has_past, uint64_t *out, size_t cap);
/* add_noop (sequential.rs:38-42, do_add_noop :106-123) */
size_t fo_keydeps_add_noop(fo_keydeps *kd, uint64_t dot, uint64_t *out,
                           size_t cap);
/* cmd_deps / noop_deps (test-only queries, sequential.rs:44-58) */
size_t fo_keydeps_cmd_deps(const fo_keydeps *kd, const uint64_t *keys,
                           size_t nkeys, uint64_t *out, size_t cap);
size_t fo_keydeps_noop_deps(const fo_keydeps *kd, uint64_t *out, size_t cap);

/* Whole-stream driver: one SequentialKeyDeps, commands in stream order.
 * is_noop may be NULL.  Output CSR (out_off[n+1], out_dep) must be sized by
 * the caller; out_dep_cap is checked.  Returns total deps or (size_t)-1 on
 * capacity overflow. */
size_t fo_keydeps_run(uint64_t shard_id, size_t n, const uint64_t *dot,
                      const uint32_t *key_off, const uint64_t *keys,
                      const uint8_t *is_noop, uint32_t *out_off,
                      uint64_t *out_dep, size_t out_dep_cap);

/* ---------------------------------------------------------------------
 * LockedKeyDeps (deps/keys/locked.rs:10-186), applied sequentially: per key
 * a read depends on the latest write and becomes the latest read; a write
 * depends on the latest read and write and becomes the latest write; noops
 * see every key's latest read and write.  Parity: the write rules are pinned
 * by key_deps_flow::<LockedKeyDeps> (keys/mod.rs:86-88, write-only); the
 * reference has no read-only known-answer test, so the read rules are
 * restated from locked.rs:100-106 and checked by hand-derived cases
 * (tests/test_oracle_rw.py).
 * ------------------------------------------------------------------- */
typedef struct fo_lkeydeps fo_lkeydeps;

fo_lkeydeps *fo_lkeydeps_new(uint64_t shard_id);
void fo_lkeydeps_free(fo_lkeydeps *kd);
size_t fo_lkeydeps_add_cmd(fo_lkeydeps *kd, uint64_t dot, const uint64_t *keys,
                           size_t nkeys, int read_only, const uint64_t *past,
                           size_t npast, int has_past, uint64_t *out, size_t cap);
size_t fo_lkeydeps_add_noop(fo_lkeydeps *kd, uint64_t dot, uint64_t *out,
                            size_t cap);
size_t fo_lkeydeps_cmd_deps(const fo_lkeydeps *kd, const uint64_t *keys,
                            size_t nkeys, uint64_t *out, size_t cap);
size_t fo_lkeydeps_noop_deps(const fo_lkeydeps *kd, uint64_t *out, size_t cap);

/* ---------------------------------------------------------------------
 * QuorumDeps  (deps/quorum.rs:7-98)
 * reports: nrep dep-sets given as CSR (rep_off[nrep+1], rep_dep).
 * Returns union size, writes sorted union into out; *flag receives the
 * boolean of check_threshold_union(threshold) (mode 0) or check_union
 * (mode 1).
 * ------------------------------------------------------------------- */
size_t fo_quorum_deps(size_t fast_quorum_size, size_t nrep,
                      const uint32_t *rep_off, const uint64_t *rep_dep,
                      int mode, size_t threshold, uint64_t *out, size_t cap,
                      int *flag);

/* ---------------------------------------------------------------------
 * Replica-view committed deps (Atlas / EPaxos collect phase):
 *   atlas.rs:214-252 (submit: coordinator add_cmd(None)),
 *   atlas.rs:255-328 (MCollect at fast-quorum members: add_cmd(past)),
 *   atlas.rs:331-397 + quorum.rs:46-64 (union of reports),
 *   epaxos.rs:203-342 (same, self report not counted, check_union).
 * Each command i has a fast quorum given by fq_proc[i*fq + j] (j=0 is the
 * coordinator) and per-member event time fq_time[i*fq + j]; every replica
 * processes the commands it belongs to in increasing (time, i) order.
 * protocol: 0 = Atlas (coordinator's own report counted), 1 = EPaxos.
 * Output: committed deps CSR (sorted per command).
 * ------------------------------------------------------------------- */
size_t fo_views_run(int protocol, uint32_t nproc, size_t n, uint32_t fq,
                    const uint64_t *dot, const uint32_t *key_off,
                    const uint64_t *keys, const uint8_t *fq_proc,
                    const uint64_t *fq_time, uint32_t *out_off,
                    uint64_t *out_dep, size_t out_dep_cap);

/* ---------------------------------------------------------------------
 * DependencyGraph + TarjanSCCFinder (executor/graph/mod.rs:45-679,
 * tarjan.rs:25-359, index.rs:145-211), AEClock executed set.
 * ------------------------------------------------------------------- */
typedef struct fo_graph fo_graph;

fo_graph *fo_graph_new(uint32_t process_id, uint64_t shard_id, uint32_t n,
                       uint32_t f, uint32_t shard_count);
void fo_graph_free(fo_graph *g);
/* handle_add (mod.rs:215-277).  Returns number of commands that became
 * ready (to_execute growth). */
size_t fo_graph_add(fo_graph *g, uint64_t dot, const uint64_t *keys,
                    size_t nkeys, const uint64_t *deps, size_t ndeps);
/* Index a vertex without searching (used by sccs_found_and_missing_dep,
 * mod.rs:1166-1308). */
void fo_graph_index_only(fo_graph *g, uint64_t dot, const uint64_t *keys,
                         size_t nkeys, const uint64_t *deps, size_t ndeps);
/* Set the executed clock frontier of `source` (util::vclock / AEClock::from,
 * mod.rs:1310-1317). */
void fo_graph_set_executed_frontier(fo_graph *g, uint32_t source,
                                    uint64_t seq);
/* find_scc(first_find, dot) (mod.rs:411-488), the "search only" entry used
 * by sccs_found_and_missing_dep.  Returns the FinderInfo kind:
 * 0 Found, 1 MissingDependencies, 2 NotPending; *ready = total_scc_count,
 * *nfound = dots moved to to_execute, missing dots written to missing. */
int fo_graph_find_scc(fo_graph *g, int first_find, uint64_t dot,
                      size_t *ready, size_t *nfound, uint64_t *missing,
                      size_t missing_cap, size_t *nmissing);
int fo_graph_executed(const fo_graph *g, uint64_t dot);

/* Drain the to_execute queue (command_to_execute, mod.rs:133-135).  For
 * every drained command writes its dot and the label of its SCC (min dot of
 * the SCC).  Returns number drained (<= cap). */
size_t fo_graph_drain(fo_graph *g, uint64_t *dots, uint64_t *scc_label,
                      size_t cap);
size_t fo_graph_pending_count(const fo_graph *g);

/* Partial replication (executor/graph/mod.rs:139-157, 168-179, 279-408;
 * index.rs:171-205).  One graph plays both executor roles of its shard, as
 * the reference's executors 0 and 1 share the VertexIndex (index.rs:21); its
 * executed clock is the main role's (Executed notifications delivered
 * before the next request).  Masks: bit s = shard s; 0 = None (a noop). */
size_t fo_graph_add_sharded(fo_graph *g, uint64_t dot, const uint64_t *keys, size_t nkeys,
                            uint64_t cmask, const uint64_t *deps, const uint64_t *dmasks,
                            size_t ndeps);
void fo_graph_handle_requests(fo_graph *g, uint64_t from, const uint64_t *dots, size_t n);
void fo_graph_cleanup(fo_graph *g);
size_t fo_graph_requests(fo_graph *g, uint64_t *shard, uint64_t *dot, size_t cap);
void fo_graph_replies_size(const fo_graph *g, size_t *nr, size_t *nd);
void fo_graph_replies_take(fo_graph *g, uint64_t *to, uint64_t *kind, uint64_t *dot,
                           uint64_t *cmask, uint64_t *doff, uint64_t *ddot, uint64_t *dmask);
size_t fo_graph_mark_executed(fo_graph *g, uint64_t dot);
int fo_graph_violation(const fo_graph *g);

/* Whole-stream driver: GraphExecutor::handle(Add) for every command in
 * arrival order, followed by fetch_commands_to_execute + execute (executor.rs:
 * 76-100, 133-145, 191-196); per-key ExecutionOrderMonitor (monitor.rs:20-28).
 * Outputs (all caller-sized to n / nkeys):
 *   exec_dot[n]   global execution order (drain order), exec_count returned
 *   scc_label[n]  per executed position, min dot of its SCC
 *   key_seq_off[K+1], key_seq[total keys]: per-key execution sequence for
 *                 key ids 0..K-1 (dense).
 * Returns number of executed commands. */
size_t fo_graph_run(uint32_t process_id, uint32_t n, uint32_t f, size_t ncmd,
                    const uint64_t *dot, const uint32_t *key_off,
                    const uint64_t *keys, const uint32_t *dep_off,
                    const uint64_t *deps, uint64_t *exec_dot,
                    uint64_t *scc_label, uint64_t key_space,
                    uint32_t *key_seq_off, uint64_t *key_seq);

/* ---------------------------------------------------------------------
 * PredecessorsGraph -- Caesar's executor (executor/pred/mod.rs:26-352,
 * index.rs).  Clocks are packed (seq << 8) | process_id, which orders like
 * Clock's derived Ord (protocol/common/pred/clocks/mod.rs:15-30).
 * ------------------------------------------------------------------- */
typedef struct fo_pred fo_pred;

fo_pred *fo_pred_new(uint32_t process_id);
void fo_pred_free(fo_pred *p);
/* add(dot, cmd, clock, deps) (mod.rs:89-130).  Returns the number of
 * commands that became ready. */
size_t fo_pred_add(fo_pred *p, uint64_t dot, uint64_t clock, const uint64_t *deps,
                   size_t ndeps);
/* command_to_execute (mod.rs:71-73), in order. */
size_t fo_pred_drain(fo_pred *p, uint64_t *dots, size_t cap);
size_t fo_pred_pending_count(const fo_pred *p);

#ifdef __cplusplus
}
#endif
#endif
