/*
 * oracle.c -- CPU restatement of fantoch's dependency hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Never linked into, loaded by or
 * called from the product library (fantoch_amd/libfantoch_hip.so).
 *
 * Every function cites the reference file:line it restates.  Hash maps and
 * sets are open-addressing tables (the reference uses hashbrown/ahash); the
 * iteration order of those containers is not part of parity.
 */
#include "oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EMPTY_KEY UINT64_MAX

static void *xmalloc(size_t n) {
  void *p = malloc(n ? n : 1);
  if (!p) {
    fprintf(stderr, "oracle: out of memory (%zu bytes)\n", n);
    abort();
  }
  return p;
}
static void *xrealloc(void *p, size_t n) {
  void *q = realloc(p, n ? n : 1);
  if (!q) {
    fprintf(stderr, "oracle: out of memory (%zu bytes)\n", n);
    abort();
  }
  return q;
}

static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

/* ------------------------------------------------------------------ */
/* u64 -> u64 map, linear probing, backward-shift deletion             */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t *k;
  uint64_t *v;
  size_t cap; /* power of two */
  size_t len;
} u64map;

static void map_init(u64map *m, size_t cap) {
  size_t c = 16;
  while (c < cap * 2) c <<= 1;
  m->cap = c;
  m->len = 0;
  m->k = (uint64_t *)xmalloc(c * sizeof(uint64_t));
  m->v = (uint64_t *)xmalloc(c * sizeof(uint64_t));
  for (size_t i = 0; i < c; i++) m->k[i] = EMPTY_KEY;
}
static void map_free(u64map *m) {
  free(m->k);
  free(m->v);
  m->k = m->v = NULL;
  m->cap = m->len = 0;
}
static void map_put(u64map *m, uint64_t key, uint64_t val);
static void map_grow(u64map *m) {
  u64map n;
  map_init(&n, m->cap);
  for (size_t i = 0; i < m->cap; i++)
    if (m->k[i] != EMPTY_KEY) map_put(&n, m->k[i], m->v[i]);
  map_free(m);
  *m = n;
}
/* returns pointer to the value slot, or NULL */
static inline uint64_t *map_get(const u64map *m, uint64_t key) {
  size_t mask = m->cap - 1;
  size_t i = mix64(key) & mask;
  for (;;) {
    uint64_t k = m->k[i];
    if (k == key) return &m->v[i];
    if (k == EMPTY_KEY) return NULL;
    i = (i + 1) & mask;
  }
}
static void map_put(u64map *m, uint64_t key, uint64_t val) {
  if ((m->len + 1) * 4 > m->cap * 3) map_grow(m);
  size_t mask = m->cap - 1;
  size_t i = mix64(key) & mask;
  for (;;) {
    uint64_t k = m->k[i];
    if (k == key) {
      m->v[i] = val;
      return;
    }
    if (k == EMPTY_KEY) {
      m->k[i] = key;
      m->v[i] = val;
      m->len++;
      return;
    }
    i = (i + 1) & mask;
  }
}
static int map_del(u64map *m, uint64_t key, uint64_t *old) {
  size_t mask = m->cap - 1;
  size_t i = mix64(key) & mask;
  for (;;) {
    uint64_t k = m->k[i];
    if (k == EMPTY_KEY) return 0;
    if (k == key) break;
    i = (i + 1) & mask;
  }
  if (old) *old = m->v[i];
  /* backward shift */
  size_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    if (m->k[j] == EMPTY_KEY) break;
    size_t h = mix64(m->k[j]) & mask;
    /* can the entry at j move to i? (h not in (i, j] cyclically) */
    int move = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
    if (move) {
      m->k[i] = m->k[j];
      m->v[i] = m->v[j];
      i = j;
    }
  }
  m->k[i] = EMPTY_KEY;
  m->len--;
  return 1;
}

/* ------------------------------------------------------------------ */
/* growable u64 vector + "HashSet<Dot>" semantics via sort-unique       */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t *a;
  size_t len, cap;
} vec64;
static void vpush(vec64 *v, uint64_t x) {
  if (v->len == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 8;
    v->a = (uint64_t *)xrealloc(v->a, v->cap * sizeof(uint64_t));
  }
  v->a[v->len++] = x;
}
static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return (x > y) - (x < y);
}
static size_t sort_unique(uint64_t *a, size_t n) {
  if (n < 2) return n;
  /* tiny sets: insertion sort */
  if (n <= 16) {
    for (size_t i = 1; i < n; i++) {
      uint64_t x = a[i];
      size_t j = i;
      while (j > 0 && a[j - 1] > x) {
        a[j] = a[j - 1];
        j--;
      }
      a[j] = x;
    }
  } else {
    qsort(a, n, sizeof(uint64_t), cmp_u64);
  }
  size_t w = 1;
  for (size_t i = 1; i < n; i++)
    if (a[i] != a[w - 1]) a[w++] = a[i];
  return w;
}
static size_t emit(const uint64_t *src, size_t n, uint64_t *out, size_t cap) {
  if (out) memcpy(out, src, (n < cap ? n : cap) * sizeof(uint64_t));
  return n;
}

/* ------------------------------------------------------------------ */
/* SequentialKeyDeps (deps/keys/sequential.rs)                          */
/* ------------------------------------------------------------------ */
struct fo_keydeps {
  uint64_t shard_id;
  u64map latest;      /* latest_deps: Key -> Dependency (dot)  :10 */
  uint64_t noop_dot;  /* noop_latest_dep (0 == None)           :11 */
  vec64 scratch;
};

fo_keydeps *fo_keydeps_new(uint64_t shard_id) {
  fo_keydeps *kd = (fo_keydeps *)calloc(1, sizeof(*kd));
  kd->shard_id = shard_id;
  map_init(&kd->latest, 1024);
  return kd;
}
void fo_keydeps_free(fo_keydeps *kd) {
  if (!kd) return;
  map_free(&kd->latest);
  free(kd->scratch.a);
  free(kd);
}

/* maybe_add_noop_latest  sequential.rs:66-70 */
static void maybe_add_noop_latest(const fo_keydeps *kd, vec64 *deps) {
  if (kd->noop_dot) vpush(deps, kd->noop_dot);
}

/* do_add_cmd  sequential.rs:72-104 */
static void do_add_cmd(fo_keydeps *kd, uint64_t dot, const uint64_t *keys,
                       size_t nkeys, vec64 *deps) {
  for (size_t i = 0; i < nkeys; i++) {
    uint64_t *slot = map_get(&kd->latest, keys[i]);
    if (slot) {
      /* previous latest is a dependency; set self as new latest  :84-89 */
      vpush(deps, *slot);
      *slot = dot;
    } else {
      map_put(&kd->latest, keys[i], dot); /* :90-95 */
    }
  }
  maybe_add_noop_latest(kd, deps); /* :100 */
}

size_t fo_keydeps_add_cmd(fo_keydeps *kd, uint64_t dot, const uint64_t *keys,
                          size_t nkeys, const uint64_t *past, size_t npast,
                          int has_past, uint64_t *out, size_t cap) {
  vec64 *d = &kd->scratch;
  d->len = 0;
  if (has_past) /* sequential.rs:31-34: start with past */
    for (size_t i = 0; i < npast; i++) vpush(d, past[i]);
  do_add_cmd(kd, dot, keys, nkeys, d);
  size_t n = sort_unique(d->a, d->len);
  return emit(d->a, n, out, cap);
}

/* do_noop_deps  sequential.rs:125-132 */
static void do_noop_deps(const fo_keydeps *kd, vec64 *deps) {
  for (size_t i = 0; i < kd->latest.cap; i++)
    if (kd->latest.k[i] != EMPTY_KEY) vpush(deps, kd->latest.v[i]);
}

/* do_add_noop  sequential.rs:106-123 */
size_t fo_keydeps_add_noop(fo_keydeps *kd, uint64_t dot, uint64_t *out,
                           size_t cap) {
  vec64 *d = &kd->scratch;
  d->len = 0;
  uint64_t prev = kd->noop_dot;
  kd->noop_dot = dot;
  if (prev) vpush(d, prev);
  do_noop_deps(kd, d);
  size_t n = sort_unique(d->a, d->len);
  return emit(d->a, n, out, cap);
}

/* cmd_deps  sequential.rs:44-50, do_cmd_deps :134-143 */
size_t fo_keydeps_cmd_deps(const fo_keydeps *kd, const uint64_t *keys,
                           size_t nkeys, uint64_t *out, size_t cap) {
  vec64 d = {0};
  maybe_add_noop_latest(kd, &d);
  for (size_t i = 0; i < nkeys; i++) {
    uint64_t *slot = map_get(&kd->latest, keys[i]);
    if (slot) vpush(&d, *slot);
  }
  size_t n = sort_unique(d.a, d.len);
  emit(d.a, n, out, cap);
  free(d.a);
  return n;
}

/* noop_deps  sequential.rs:52-58 */
size_t fo_keydeps_noop_deps(const fo_keydeps *kd, uint64_t *out, size_t cap) {
  vec64 d = {0};
  maybe_add_noop_latest(kd, &d);
  do_noop_deps(kd, &d);
  size_t n = sort_unique(d.a, d.len);
  emit(d.a, n, out, cap);
  free(d.a);
  return n;
}

size_t fo_keydeps_run(uint64_t shard_id, size_t n, const uint64_t *dot,
                      const uint32_t *key_off, const uint64_t *keys,
                      const uint8_t *is_noop, uint32_t *out_off,
                      uint64_t *out_dep, size_t out_dep_cap) {
  fo_keydeps *kd = fo_keydeps_new(shard_id);
  size_t total = 0;
  out_off[0] = 0;
  for (size_t i = 0; i < n; i++) {
    size_t room = out_dep_cap > total ? out_dep_cap - total : 0;
    size_t c;
    if (is_noop && is_noop[i])
      c = fo_keydeps_add_noop(kd, dot[i], out_dep + total, room);
    else
      c = fo_keydeps_add_cmd(kd, dot[i], keys + key_off[i],
                             key_off[i + 1] - key_off[i], NULL, 0, 0,
                             out_dep + total, room);
    if (c > room) {
      fo_keydeps_free(kd);
      return (size_t)-1;
    }
    total += c;
    out_off[i + 1] = (uint32_t)total;
  }
  fo_keydeps_free(kd);
  return total;
}

/* ------------------------------------------------------------------ */
/* LockedKeyDeps (deps/keys/locked.rs), applied sequentially           */
/* ------------------------------------------------------------------ */
struct fo_lkeydeps {
  u64map w, r;        /* LatestRW{read, write} per key  :10-15 */
  uint64_t noop_dot;  /* latest_noop (0 == None)        :21 */
  vec64 scratch;
};

fo_lkeydeps *fo_lkeydeps_new(uint64_t shard_id) {
  fo_lkeydeps *kd = (fo_lkeydeps *)calloc(1, sizeof(*kd));
  (void)shard_id;
  map_init(&kd->w, 1024);
  map_init(&kd->r, 1024);
  return kd;
}
void fo_lkeydeps_free(fo_lkeydeps *kd) {
  if (!kd) return;
  map_free(&kd->w);
  map_free(&kd->r);
  free(kd->scratch.a);
  free(kd);
}

/* add_cmd (:34-46) -> do_add_cmd (:83-128) */
size_t fo_lkeydeps_add_cmd(fo_lkeydeps *kd, uint64_t dot, const uint64_t *keys,
                           size_t nkeys, int read_only, const uint64_t *past,
                           size_t npast, int has_past, uint64_t *out, size_t cap) {
  vec64 *d = &kd->scratch;
  d->len = 0;
  if (has_past)
    for (size_t i = 0; i < npast; i++) vpush(d, past[i]);
  for (size_t i = 0; i < nkeys; i++) {
    uint64_t *wd = map_get(&kd->w, keys[i]);
    if (read_only) { /* :100-106: latest write; become the latest read */
      if (wd) vpush(d, *wd);
      map_put(&kd->r, keys[i], dot);
    } else { /* :107-117: latest read and write; become the latest write */
      uint64_t *rd = map_get(&kd->r, keys[i]);
      if (rd) vpush(d, *rd);
      if (wd) {
        vpush(d, *wd);
        *wd = dot;
      } else {
        map_put(&kd->w, keys[i], dot);
      }
    }
  }
  if (kd->noop_dot) vpush(d, kd->noop_dot); /* :124 */
  size_t n = sort_unique(d->a, d->len);
  return emit(d->a, n, out, cap);
}

/* do_noop_deps (:156-169): every key's latest read and write */
static void lk_noop_deps(const fo_lkeydeps *kd, vec64 *d) {
  for (size_t i = 0; i < kd->w.cap; i++)
    if (kd->w.k[i] != EMPTY_KEY) vpush(d, kd->w.v[i]);
  for (size_t i = 0; i < kd->r.cap; i++)
    if (kd->r.k[i] != EMPTY_KEY) vpush(d, kd->r.v[i]);
}

/* add_noop (:48-52) -> do_add_noop (:130-154) */
size_t fo_lkeydeps_add_noop(fo_lkeydeps *kd, uint64_t dot, uint64_t *out, size_t cap) {
  vec64 *d = &kd->scratch;
  d->len = 0;
  uint64_t prev = kd->noop_dot;
  kd->noop_dot = dot;
  if (prev) vpush(d, prev);
  lk_noop_deps(kd, d);
  size_t n = sort_unique(d->a, d->len);
  return emit(d->a, n, out, cap);
}

/* cmd_deps (:54-60) with do_cmd_deps (:172-185) */
size_t fo_lkeydeps_cmd_deps(const fo_lkeydeps *kd, const uint64_t *keys, size_t nkeys,
                            uint64_t *out, size_t cap) {
  vec64 d = {0};
  if (kd->noop_dot) vpush(&d, kd->noop_dot);
  for (size_t i = 0; i < nkeys; i++) {
    uint64_t *rd = map_get(&kd->r, keys[i]);
    uint64_t *wd = map_get(&kd->w, keys[i]);
    if (rd) vpush(&d, *rd);
    if (wd) vpush(&d, *wd);
  }
  size_t n = sort_unique(d.a, d.len);
  emit(d.a, n, out, cap);
  free(d.a);
  return n;
}

/* noop_deps (:62-68) */
size_t fo_lkeydeps_noop_deps(const fo_lkeydeps *kd, uint64_t *out, size_t cap) {
  vec64 d = {0};
  if (kd->noop_dot) vpush(&d, kd->noop_dot);
  lk_noop_deps(kd, &d);
  size_t n = sort_unique(d.a, d.len);
  emit(d.a, n, out, cap);
  free(d.a);
  return n;
}

/* ------------------------------------------------------------------ */
/* QuorumDeps (deps/quorum.rs)                                         */
/* ------------------------------------------------------------------ */
size_t fo_quorum_deps(size_t fast_quorum_size, size_t nrep,
                      const uint32_t *rep_off, const uint64_t *rep_dep,
                      int mode, size_t threshold, uint64_t *out, size_t cap,
                      int *flag) {
  /* add :28-38 (count per dep) */
  u64map counts;
  map_init(&counts, 64);
  for (size_t r = 0; r < nrep; r++)
    for (uint32_t j = rep_off[r]; j < rep_off[r + 1]; j++) {
      uint64_t *c = map_get(&counts, rep_dep[j]);
      if (c)
        (*c)++;
      else
        map_put(&counts, rep_dep[j], 1);
    }
  vec64 u = {0};
  int eq = 1;
  if (mode == 0) {
    /* check_threshold_union :46-64 */
    for (size_t i = 0; i < counts.cap; i++)
      if (counts.k[i] != EMPTY_KEY) {
        eq = eq && counts.v[i] >= threshold;
        vpush(&u, counts.k[i]);
      }
  } else {
    /* check_union :67-98: equal iff a single distinct count == fq size */
    uint64_t seen = 0;
    int distinct = 0;
    for (size_t i = 0; i < counts.cap; i++)
      if (counts.k[i] != EMPTY_KEY) {
        vpush(&u, counts.k[i]);
        if (distinct == 0) {
          seen = counts.v[i];
          distinct = 1;
        } else if (counts.v[i] != seen) {
          distinct = 2;
        }
      }
    eq = distinct == 0 ? 1 : (distinct == 1 ? seen == fast_quorum_size : 0);
  }
  size_t n = sort_unique(u.a, u.len);
  emit(u.a, n, out, cap);
  free(u.a);
  map_free(&counts);
  if (flag) *flag = eq;
  return n;
}

/* ------------------------------------------------------------------ */
/* Replica views: per-replica SequentialKeyDeps + union of reports     */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t time;
  uint32_t cmd;
  uint32_t slot; /* 0 = coordinator */
} view_event;

static int cmp_event(const void *a, const void *b) {
  const view_event *x = (const view_event *)a, *y = (const view_event *)b;
  if (x->time != y->time) return (x->time > y->time) - (x->time < y->time);
  if (x->cmd != y->cmd) return (x->cmd > y->cmd) - (x->cmd < y->cmd);
  return (x->slot > y->slot) - (x->slot < y->slot);
}

size_t fo_views_run(int protocol, uint32_t nproc, size_t n, uint32_t fq,
                    const uint64_t *dot, const uint32_t *key_off,
                    const uint64_t *keys, const uint8_t *fq_proc,
                    const uint64_t *fq_time, uint32_t *out_off,
                    uint64_t *out_dep, size_t out_dep_cap) {
  (void)protocol; /* Atlas counts the coordinator's own report
                     (atlas.rs:236,291-301), EPaxos does not (epaxos.rs:668),
                     but every member report includes the coordinator's deps
                     as `past` (atlas.rs:303-309, epaxos.rs:275-281), so the
                     union is identical. */
  fo_keydeps **kd = (fo_keydeps **)xmalloc((nproc + 1) * sizeof(*kd));
  for (uint32_t p = 0; p <= nproc; p++) kd[p] = fo_keydeps_new(0);
  size_t nev = n * fq;
  view_event *ev = (view_event *)xmalloc(nev * sizeof(view_event));
  for (size_t i = 0; i < n; i++)
    for (uint32_t j = 0; j < fq; j++) {
      ev[i * fq + j].time = fq_time[i * fq + j];
      ev[i * fq + j].cmd = (uint32_t)i;
      ev[i * fq + j].slot = j;
    }
  qsort(ev, nev, sizeof(view_event), cmp_event);
  /* coordinator deps (past for members) and per-command union */
  vec64 *coord = (vec64 *)calloc(n, sizeof(vec64));
  vec64 *uni = (vec64 *)calloc(n, sizeof(vec64));
  uint8_t *coord_done = (uint8_t *)calloc(n, 1);

  for (size_t e = 0; e < nev; e++) {
    uint32_t i = ev[e].cmd, j = ev[e].slot;
    uint32_t p = fq_proc[(size_t)i * fq + j];
    const uint64_t *ks = keys + key_off[i];
    size_t nk = key_off[i + 1] - key_off[i];
    if (j == 0) {
      /* handle_submit: add_cmd(dot, cmd, None)  atlas.rs:236 */
      size_t c = fo_keydeps_add_cmd(kd[p], dot[i], ks, nk, NULL, 0, 0, NULL, 0);
      /* add_cmd leaves its sorted result in the instance's scratch vector */
      coord[i].len = 0;
      for (size_t t = 0; t < c; t++) vpush(&coord[i], kd[p]->scratch.a[t]);
      coord_done[i] = 1;
      for (size_t t = 0; t < coord[i].len; t++) vpush(&uni[i], coord[i].a[t]);
    } else {
      /* handle_mcollect at a fast-quorum member: add_cmd(past = coord deps)
       * atlas.rs:303-309.  Event times guarantee the coordinator ran first. */
      if (!coord_done[i]) {
        fprintf(stderr, "oracle: member event before coordinator (cmd %u)\n",
                i);
        abort();
      }
      size_t c = fo_keydeps_add_cmd(kd[p], dot[i], ks, nk, coord[i].a,
                                    coord[i].len, 1, NULL, 0);
      for (size_t t = 0; t < c; t++) vpush(&uni[i], kd[p]->scratch.a[t]);
    }
  }
  size_t total = 0;
  out_off[0] = 0;
  int overflow = 0;
  for (size_t i = 0; i < n; i++) {
    size_t c = sort_unique(uni[i].a, uni[i].len);
    if (total + c > out_dep_cap) overflow = 1;
    if (!overflow) memcpy(out_dep + total, uni[i].a, c * sizeof(uint64_t));
    total += c;
    out_off[i + 1] = (uint32_t)total;
    free(uni[i].a);
    free(coord[i].a);
  }
  free(uni);
  free(coord);
  free(coord_done);

  free(ev);
  for (uint32_t p = 0; p <= nproc; p++) fo_keydeps_free(kd[p]);
  free(kd);
  return overflow ? (size_t)-1 : total;
}

/* ------------------------------------------------------------------ */
/* AEClock<ProcessId> (threshold crate): contiguous frontier + exceptions */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t frontier[256];
  u64map exc; /* key = packed dot */
} aeclock;

static void ae_init(aeclock *c) {
  memset(c->frontier, 0, sizeof(c->frontier));
  map_init(&c->exc, 64);
}
static inline int ae_contains(const aeclock *c, uint64_t dot) {
  uint64_t s = FO_SEQ(dot);
  if (s <= c->frontier[FO_SRC(dot)]) return 1;
  return c->exc.len && map_get(&c->exc, dot) != NULL;
}
static void ae_add(aeclock *c, uint64_t dot) {
  uint32_t src = FO_SRC(dot);
  uint64_t s = FO_SEQ(dot);
  if (s <= c->frontier[src]) return;
  if (s == c->frontier[src] + 1) {
    c->frontier[src] = s;
    /* absorb exceptions */
    while (c->exc.len) {
      uint64_t nd = FO_DOT(src, c->frontier[src] + 1);
      if (!map_del(&c->exc, nd, NULL)) break;
      c->frontier[src]++;
    }
  } else {
    map_put(&c->exc, dot, 1);
  }
}

/* ------------------------------------------------------------------ */
/* DependencyGraph + TarjanSCCFinder                                    */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t dot;
  uint64_t keys_at; /* offset in key pool */
  uint32_t nkeys;
  uint64_t deps_at; /* offset in dep pool (dep masks at the same offsets) */
  uint32_t ndeps;
  uint64_t cmask;   /* Command::shards() as a bitmask (command.rs:103-110) */
  uint64_t id, low; /* tarjan.rs:329-331 */
  uint8_t on_stack;
  uint8_t alive;
} vertex;

typedef struct {
  uint64_t child;
  int64_t next;
} pend_node;

typedef struct {
  uint64_t dot;
  uint64_t label;
} exec_item;

struct fo_graph {
  uint32_t process_id, n, f, shard_count;
  uint64_t shard_id;
  aeclock executed;          /* mod.rs:50 */
  u64map vindex;             /* VertexIndex: dot -> vertex slot, index.rs */
  vertex *vs;
  size_t nvs, capvs;
  uint64_t *kpool;
  size_t nk, capk;
  uint64_t *dpool;
  uint64_t *mpool;           /* Dependency::shards bitmask of each dpool entry
                                (0 = None, a noop) */
  size_t nd, capd;
  u64map pindex;             /* PendingIndex: dot -> head node, index.rs:145 */
  /* partial replication (graph/mod.rs:139-157, 168-179, 279-408) */
  u64map depmask;            /* dep dot -> its Dependency::shards bitmask */
  vec64 req_shard, req_dot;  /* out_requests, not yet taken (mod.rs:147-150) */
  vec64 buf_from, buf_dot;   /* buffered_in_requests (mod.rs:363-371) */
  vec64 rep_to, rep_kind, rep_dot, rep_cmask, rep_doff; /* out_request_replies */
  vec64 rep_ddot, rep_dmask;
  int violation;             /* an invariant the reference panics on */
  pend_node *pnodes;
  size_t npn, cappn;
  /* finder state tarjan.rs:26-34 */
  uint64_t fid;
  vec64 stack;
  vec64 sccs_flat; /* members of found SCCs (each SCC sorted) */
  vec64 scc_ends;  /* end offsets into sccs_flat */
  vec64 missing;   /* missing_deps set */
  /* to_execute queue mod.rs:60 */
  exec_item *q;
  size_t qhead, qtail, qcap;
  /* recursion emulation */
  struct frame {
    size_t v;
    uint32_t i;
    size_t mdc;
  } *frames;
  size_t nframes, capframes;
};

fo_graph *fo_graph_new(uint32_t process_id, uint64_t shard_id, uint32_t n,
                       uint32_t f, uint32_t shard_count) {
  fo_graph *g = (fo_graph *)calloc(1, sizeof(*g));
  g->process_id = process_id;
  g->shard_id = shard_id;
  g->n = n;
  g->f = f;
  g->shard_count = shard_count ? shard_count : 1;
  ae_init(&g->executed);
  map_init(&g->vindex, 1024);
  map_init(&g->pindex, 256);
  map_init(&g->depmask, 256);
  return g;
}

void fo_graph_free(fo_graph *g) {
  if (!g) return;
  map_free(&g->executed.exc);
  map_free(&g->vindex);
  map_free(&g->pindex);
  map_free(&g->depmask);
  free(g->vs);
  free(g->kpool);
  free(g->dpool);
  free(g->mpool);
  free(g->req_shard.a);
  free(g->req_dot.a);
  free(g->buf_from.a);
  free(g->buf_dot.a);
  free(g->rep_to.a);
  free(g->rep_kind.a);
  free(g->rep_dot.a);
  free(g->rep_cmask.a);
  free(g->rep_doff.a);
  free(g->rep_ddot.a);
  free(g->rep_dmask.a);
  free(g->pnodes);
  free(g->stack.a);
  free(g->sccs_flat.a);
  free(g->scc_ends.a);
  free(g->missing.a);
  free(g->q);
  free(g->frames);
  free(g);
}

static size_t new_vertex(fo_graph *g, uint64_t dot, const uint64_t *keys,
                         size_t nkeys, const uint64_t *deps, size_t ndeps,
                         uint64_t cmask, const uint64_t *dmasks) {
  if (g->nvs == g->capvs) {
    g->capvs = g->capvs ? g->capvs * 2 : 1024;
    g->vs = (vertex *)xrealloc(g->vs, g->capvs * sizeof(vertex));
  }
  while (g->nk + nkeys > g->capk) {
    g->capk = g->capk ? g->capk * 2 : 4096;
    g->kpool = (uint64_t *)xrealloc(g->kpool, g->capk * sizeof(uint64_t));
  }
  while (g->nd + ndeps > g->capd) {
    g->capd = g->capd ? g->capd * 2 : 4096;
    g->dpool = (uint64_t *)xrealloc(g->dpool, g->capd * sizeof(uint64_t));
    g->mpool = (uint64_t *)xrealloc(g->mpool, g->capd * sizeof(uint64_t));
  }
  vertex *v = &g->vs[g->nvs];
  v->dot = dot;
  v->keys_at = g->nk;
  v->nkeys = (uint32_t)nkeys;
  if (nkeys) memcpy(g->kpool + g->nk, keys, nkeys * sizeof(uint64_t));
  g->nk += nkeys;
  v->deps_at = g->nd;
  v->ndeps = (uint32_t)ndeps;
  if (ndeps) memcpy(g->dpool + g->nd, deps, ndeps * sizeof(uint64_t));
  for (size_t i = 0; i < ndeps; i++) {
    g->mpool[g->nd + i] = dmasks ? dmasks[i] : 0;
    if (dmasks) map_put(&g->depmask, deps[i], dmasks[i]);
  }
  g->nd += ndeps;
  v->cmask = cmask;
  v->id = v->low = 0;
  v->on_stack = 0;
  v->alive = 1;
  return g->nvs++;
}

/* VertexIndex::index  index.rs:33-37; panics on double index mod.rs:235 */
static size_t index_vertex(fo_graph *g, uint64_t dot, const uint64_t *keys,
                           size_t nkeys, const uint64_t *deps, size_t ndeps,
                           uint64_t cmask, const uint64_t *dmasks) {
  if (map_get(&g->vindex, dot)) {
    fprintf(stderr, "oracle: Graph::handle_add tried to index already indexed "
                    "dot (%u,%llu)\n",
            FO_SRC(dot), (unsigned long long)FO_SEQ(dot));
    abort();
  }
  size_t slot = new_vertex(g, dot, keys, nkeys, deps, ndeps, cmask, dmasks);
  map_put(&g->vindex, dot, slot);
  return slot;
}

static inline vertex *find_vertex(const fo_graph *g, uint64_t dot) {
  uint64_t *s = map_get(&g->vindex, dot);
  return s ? &g->vs[*s] : NULL;
}

static void push_frame(fo_graph *g, size_t v) {
  if (g->nframes == g->capframes) {
    g->capframes = g->capframes ? g->capframes * 2 : 256;
    g->frames = (struct frame *)xrealloc(g->frames,
                                         g->capframes * sizeof(struct frame));
  }
  g->frames[g->nframes].v = v;
  g->frames[g->nframes].i = 0;
  g->frames[g->nframes].mdc = 0;
  g->nframes++;
}

enum { FR_FOUND = 0, FR_MISSING = 1, FR_NOTPENDING = 2, FR_NOTFOUND = 3 };

/* enter strong_connect for vertex slot v  tarjan.rs:110-122 */
static void sc_enter(fo_graph *g, size_t v) {
  g->fid++;
  vertex *x = &g->vs[v];
  x->id = g->fid;
  x->low = g->fid;
  x->on_stack = 1;
  vpush(&g->stack, x->dot);
  push_frame(g, v);
}

/* TarjanSCCFinder::strong_connect  tarjan.rs:98-319, recursion emulated with
 * an explicit frame stack.  Returns FR_FOUND / FR_MISSING / FR_NOTFOUND;
 * on FR_MISSING the missing dependency is left in *missing_dep.
 * *root_mdc receives the root's missing_deps_count. */
static int strong_connect(fo_graph *g, int first_find, size_t root,
                          size_t *scc_count, size_t *root_mdc,
                          uint64_t *missing_dep) {
  g->nframes = 0;
  sc_enter(g, root);
  int child_result = -1; /* result delivered by a just-finished child */
  size_t child_mdc = 0;
  size_t child_v = 0;
  for (;;) {
    struct frame *fr = &g->frames[g->nframes - 1];
    vertex *x = &g->vs[fr->v];
    if (child_result >= 0) {
      /* back from recursion  tarjan.rs:199-217 */
      fr->mdc += child_mdc; /* :202 */
      if (child_result == FR_MISSING) {
        /* give up: propagate MissingDependencies to the root  :205-207 */
        g->nframes--;
        if (g->nframes == 0) {
          *root_mdc = fr->mdc;
          return FR_MISSING;
        }
        child_mdc = fr->mdc;
        child_result = FR_MISSING;
        continue;
      }
      vertex *c = &g->vs[child_v];
      if (c->low < x->low) x->low = c->low; /* :214 */
      child_result = -1;
    }
    if (fr->i < x->ndeps) {
      uint64_t dep = g->dpool[x->deps_at + fr->i];
      fr->i++;
      /* ignore self or executed  :131-148 */
      if (dep == x->dot || ae_contains(&g->executed, dep)) continue;
      vertex *d = find_vertex(g, dep);
      if (!d) {
        /* missing dependency  :151-170 */
        if (g->shard_count == 1 || !first_find) {
          *missing_dep = dep;
          /* return MissingDependencies from this frame upwards */
          g->nframes--;
          if (g->nframes == 0) {
            *root_mdc = fr->mdc;
            return FR_MISSING;
          }
          child_mdc = fr->mdc;
          child_result = FR_MISSING;
          continue;
        }
        vpush(&g->missing, dep);
        fr->mdc++;
        continue;
      }
      if (d->id == 0) {
        /* not visited: recurse  :176-217 */
        sc_enter(g, (size_t)(d - g->vs));
        continue;
      }
      if (d->on_stack && d->id < x->low) x->low = d->id; /* :220-224 */
      continue;
    }
    /* all deps visited  :233-318 */
    int result;
    if (fr->mdc == 0 && x->id == x->low) {
      size_t start = g->sccs_flat.len;
      for (;;) {
        uint64_t member = g->stack.a[--g->stack.len];
        vertex *m = find_vertex(g, member);
        (*scc_count)++;
        m->on_stack = 0;
        vpush(&g->sccs_flat, member);
        ae_add(&g->executed, member); /* :296 */
        if (member == x->dot) break;
      }
      /* SCC = BTreeSet<Dot>: sorted by dot  tarjan.rs:14-15 */
      sort_unique(g->sccs_flat.a + start, g->sccs_flat.len - start);
      vpush(&g->scc_ends, g->sccs_flat.len);
      result = FR_FOUND;
    } else {
      result = FR_NOTFOUND;
    }
    size_t done_v = fr->v;
    size_t mdc = fr->mdc;
    g->nframes--;
    if (g->nframes == 0) {
      *root_mdc = mdc;
      return result;
    }
    child_result = result;
    child_mdc = mdc;
    child_v = done_v;
  }
}

static void q_push(fo_graph *g, uint64_t dot, uint64_t label) {
  if (g->qtail == g->qcap) {
    if (g->qhead > 0) {
      memmove(g->q, g->q + g->qhead, (g->qtail - g->qhead) * sizeof(exec_item));
      g->qtail -= g->qhead;
      g->qhead = 0;
    }
    if (g->qtail == g->qcap) {
      g->qcap = g->qcap ? g->qcap * 2 : 1024;
      g->q = (exec_item *)xrealloc(g->q, g->qcap * sizeof(exec_item));
    }
  }
  g->q[g->qtail].dot = dot;
  g->q[g->qtail].label = label;
  g->qtail++;
}

/* save_scc  mod.rs:490-525: remove members from the index in dot order and
 * push them to to_execute. */
static void save_scc(fo_graph *g, const uint64_t *scc, size_t len,
                     vec64 *dots) {
  uint64_t label = scc[0]; /* min dot */
  for (size_t i = 0; i < len; i++) {
    uint64_t slot;
    if (!map_del(&g->vindex, scc[i], &slot)) {
      fprintf(stderr, "oracle: dots from an SCC should exist\n");
      abort();
    }
    g->vs[slot].alive = 0;
    vpush(dots, scc[i]);
    q_push(g, scc[i], label);
  }
}

/* finalize  tarjan.rs:60-96: reset ids of stack members, return visited */
static void finalize(fo_graph *g, vec64 *visited) {
  g->fid = 0;
  while (g->stack.len) {
    uint64_t dot = g->stack.a[--g->stack.len];
    vertex *v = find_vertex(g, dot);
    if (!v) {
      fprintf(stderr, "oracle: Finder::finalize stack member should exist\n");
      abort();
    }
    v->id = 0;
    if (visited) vpush(visited, dot);
  }
}

typedef struct {
  int kind; /* FR_FOUND / FR_MISSING (MissingDependencies) / FR_NOTPENDING */
  vec64 dots;
  vec64 visited;
  vec64 missing;
} finder_info;

static void fi_free(finder_info *fi) {
  free(fi->dots.a);
  free(fi->visited.a);
  free(fi->missing.a);
}

/* find_scc  mod.rs:411-488 */
static void find_scc(fo_graph *g, int first_find, uint64_t dot,
                     size_t *total_scc_count, finder_info *out) {
  memset(out, 0, sizeof(*out));
  vertex *v = find_vertex(g, dot);
  if (!v) { /* strong_connect wrapper mod.rs:646-671 */
    out->kind = FR_NOTPENDING;
    return;
  }
  size_t scc_count = 0, mdc = 0;
  uint64_t missing_dep = 0;
  g->sccs_flat.len = 0;
  g->scc_ends.len = 0;
  g->missing.len = 0;
  int r = strong_connect(g, first_find, (size_t)(v - g->vs), &scc_count, &mdc,
                         &missing_dep);
  *total_scc_count += scc_count;
  /* save new SCCs  :440-446 */
  size_t start = 0;
  for (size_t s = 0; s < g->scc_ends.len; s++) {
    size_t end = g->scc_ends.a[s];
    save_scc(g, g->sccs_flat.a + start, end - start, &out->dots);
    start = end;
  }
  /* finalize  :449 */
  finalize(g, &out->visited);
  size_t nm = sort_unique(g->missing.a, g->missing.len);
  switch (r) {
  case FR_FOUND:
    out->kind = FR_FOUND;
    break;
  case FR_MISSING:
    out->kind = FR_MISSING;
    vpush(&out->missing, missing_dep);
    break;
  default: /* NotFound  :479-486 */
    if (nm == 0) {
      fprintf(stderr, "oracle: either there's a missing dependency, or we "
                      "should find an SCC\n");
      abort();
    }
    out->kind = FR_MISSING;
    for (size_t i = 0; i < nm; i++) vpush(&out->missing, g->missing.a[i]);
    break;
  }
}

/* index_pending  mod.rs:527-556 -> PendingIndex::index  index.rs:171-205:
 * `dot` becomes a child of each missing dependency; the first time a
 * dependency is indexed (a vacant entry) and its shard set excludes this
 * shard, it is requested from Dot::target_shard(n) = (source - 1) / n
 * (id.rs:59-61).  "shards should be set if it's not a noop" (index.rs:
 * 190-194): a noop dependency there is an invariant violation. */
static void index_pending(fo_graph *g, uint64_t dot, const vec64 *missing) {
  for (size_t i = 0; i < missing->len; i++) {
    uint64_t parent = missing->a[i];
    if (g->npn == g->cappn) {
      g->cappn = g->cappn ? g->cappn * 2 : 256;
      g->pnodes =
          (pend_node *)xrealloc(g->pnodes, g->cappn * sizeof(pend_node));
    }
    uint64_t *head = map_get(&g->pindex, parent);
    g->pnodes[g->npn].child = dot;
    g->pnodes[g->npn].next = head ? (int64_t)*head : -1;
    if (head) {
      *head = g->npn;
    } else {
      map_put(&g->pindex, parent, g->npn);
      if (g->shard_count > 1) { /* vacant: maybe ask another shard */
        uint64_t *m = map_get(&g->depmask, parent);
        uint64_t mask = m ? *m : 0;
        if (mask == 0) {
          g->violation = 1;
        } else if (!((g->shard_id < 64) && ((mask >> g->shard_id) & 1))) {
          vpush(&g->req_shard, (FO_SRC(parent) - 1) / (g->n ? g->n : 1));
          vpush(&g->req_dot, parent);
        }
      }
    }
    g->npn++;
  }
}

static void try_pending(fo_graph *g, vec64 *pending, vec64 *dots,
                        size_t *total_scc_count);

/* check_pending  mod.rs:558-589 */
static void check_pending(fo_graph *g, vec64 *dots, size_t *total_scc_count) {
  while (dots->len) {
    uint64_t dot = dots->a[--dots->len];
    uint64_t head;
    if (map_del(&g->pindex, dot, &head)) {
      vec64 pending = {0};
      for (int64_t p = (int64_t)head; p >= 0; p = g->pnodes[p].next)
        vpush(&pending, g->pnodes[p].child);
      /* HashSet<Dot>: dedup; iterate in dot order (hash order in the
       * reference; not part of parity) */
      pending.len = sort_unique(pending.a, pending.len);
      try_pending(g, &pending, dots, total_scc_count);
      free(pending.a);
    }
  }
}

/* try_pending  mod.rs:591-644 */
static void try_pending(fo_graph *g, vec64 *pending, vec64 *dots,
                        size_t *total_scc_count) {
  u64map visited;
  map_init(&visited, 16);
  for (size_t i = 0; i < pending->len; i++) {
    uint64_t dot = pending->a[i];
    if (map_get(&visited, dot)) continue;
    finder_info fi;
    find_scc(g, 0, dot, total_scc_count, &fi);
    if (fi.kind == FR_FOUND) {
      map_free(&visited);
      map_init(&visited, 16);
      for (size_t j = 0; j < fi.dots.len; j++) vpush(dots, fi.dots.a[j]);
    } else if (fi.kind == FR_MISSING) {
      index_pending(g, dot, &fi.missing);
      if (fi.dots.len) {
        map_free(&visited);
        map_init(&visited, 16);
      } else {
        for (size_t j = 0; j < fi.visited.len; j++)
          map_put(&visited, fi.visited.a[j], 1);
      }
      for (size_t j = 0; j < fi.dots.len; j++) vpush(dots, fi.dots.a[j]);
    }
    fi_free(&fi);
  }
  map_free(&visited);
}

/* handle_add  mod.rs:215-277 */
static size_t graph_add(fo_graph *g, uint64_t dot, const uint64_t *keys, size_t nkeys,
                        uint64_t cmask, const uint64_t *deps, const uint64_t *dmasks,
                        size_t ndeps) {
  index_vertex(g, dot, keys, nkeys, deps, ndeps, cmask, dmasks);
  size_t initial_ready = g->qtail - g->qhead;
  size_t total = 0;
  finder_info fi;
  find_scc(g, 1, dot, &total, &fi);
  if (fi.kind == FR_FOUND) {
    check_pending(g, &fi.dots, &total);
  } else if (fi.kind == FR_MISSING) {
    index_pending(g, dot, &fi.missing);
    check_pending(g, &fi.dots, &total);
  } else {
    fprintf(stderr, "oracle: just added dot must be pending\n");
    abort();
  }
  fi_free(&fi);
  size_t ready = g->qtail - g->qhead;
  if (ready != initial_ready + total) { /* mod.rs:264-265 */
    fprintf(stderr, "oracle: to_execute growth mismatch\n");
    abort();
  }
  return total;
}

size_t fo_graph_add(fo_graph *g, uint64_t dot, const uint64_t *keys,
                    size_t nkeys, const uint64_t *deps, size_t ndeps) {
  return graph_add(g, dot, keys, nkeys, 0, deps, NULL, ndeps);
}

size_t fo_graph_add_sharded(fo_graph *g, uint64_t dot, const uint64_t *keys, size_t nkeys,
                            uint64_t cmask, const uint64_t *deps, const uint64_t *dmasks,
                            size_t ndeps) {
  return graph_add(g, dot, keys, nkeys, cmask, deps, dmasks, ndeps);
}

/* process_requests  mod.rs:297-375: Info{dot, cmd, deps} for an indexed
 * vertex (panic if the requester replicates it, :313-322), Executed{dot} for
 * an executed dot, otherwise buffered until the next cleanup.  Dots are
 * processed in the order given. */
static void process_requests(fo_graph *g, uint64_t from, const uint64_t *dots, size_t n) {
  for (size_t i = 0; i < n; i++) {
    uint64_t d = dots[i];
    vertex *v = find_vertex(g, d);
    if (v) {
      if (from < 64 && ((v->cmask >> from) & 1)) {
        g->violation = 1;
        continue;
      }
      vpush(&g->rep_to, from);
      vpush(&g->rep_kind, 0); /* FH_REPLY_INFO */
      vpush(&g->rep_dot, d);
      vpush(&g->rep_cmask, v->cmask);
      for (uint32_t e = 0; e < v->ndeps; e++) {
        vpush(&g->rep_ddot, g->dpool[v->deps_at + e]);
        vpush(&g->rep_dmask, g->mpool[v->deps_at + e]);
      }
      vpush(&g->rep_doff, g->rep_ddot.len);
    } else if (ae_contains(&g->executed, d)) {
      vpush(&g->rep_to, from);
      vpush(&g->rep_kind, 1); /* FH_REPLY_EXECUTED */
      vpush(&g->rep_dot, d);
      vpush(&g->rep_cmask, 0);
      vpush(&g->rep_doff, g->rep_ddot.len);
    } else {
      int dup = 0; /* HashMap<ShardId, HashSet<Dot>> */
      for (size_t b = 0; b < g->buf_dot.len && !dup; b++)
        dup = g->buf_from.a[b] == from && g->buf_dot.a[b] == d;
      if (!dup) {
        vpush(&g->buf_from, from);
        vpush(&g->buf_dot, d);
      }
    }
  }
}

/* handle_request  mod.rs:279-295 */
void fo_graph_handle_requests(fo_graph *g, uint64_t from, const uint64_t *dots, size_t n) {
  process_requests(g, from, dots, n);
}

typedef struct {
  uint64_t from, dot;
} fo_pair;
static int cmp_pair(const void *a, const void *b) {
  const fo_pair *x = (const fo_pair *)a, *y = (const fo_pair *)b;
  if (x->from != y->from) return x->from < y->from ? -1 : 1;
  return x->dot < y->dot ? -1 : x->dot > y->dot;
}

/* cleanup -> check_pending_requests  mod.rs:168-179, 673-678: the buffered
 * requests, taken, processed again (shard by shard, dots ascending: hash
 * order in the reference) */
void fo_graph_cleanup(fo_graph *g) {
  size_t n = g->buf_dot.len;
  if (!n) return;
  fo_pair *p = (fo_pair *)xmalloc(n * sizeof(fo_pair));
  for (size_t i = 0; i < n; i++) {
    p[i].from = g->buf_from.a[i];
    p[i].dot = g->buf_dot.a[i];
  }
  g->buf_from.len = g->buf_dot.len = 0;
  qsort(p, n, sizeof(fo_pair), cmp_pair);
  uint64_t *d = (uint64_t *)xmalloc(n * sizeof(uint64_t));
  for (size_t i = 0; i < n;) {
    size_t j = i;
    while (j < n && p[j].from == p[i].from) {
      d[j - i] = p[j].dot;
      j++;
    }
    process_requests(g, p[i].from, d, j - i);
    i = j;
  }
  free(d);
  free(p);
}

/* requests()  mod.rs:147-150: taken, as (target shard, dot) sorted unique */
size_t fo_graph_requests(fo_graph *g, uint64_t *shard, uint64_t *dot, size_t cap) {
  size_t n = g->req_dot.len;
  fo_pair *p = (fo_pair *)xmalloc((n ? n : 1) * sizeof(fo_pair));
  for (size_t i = 0; i < n; i++) {
    p[i].from = g->req_shard.a[i];
    p[i].dot = g->req_dot.a[i];
  }
  qsort(p, n, sizeof(fo_pair), cmp_pair);
  size_t m = 0;
  for (size_t i = 0; i < n; i++) {
    if (m && p[i].from == p[m - 1].from && p[i].dot == p[m - 1].dot) continue;
    p[m++] = p[i];
  }
  if (m <= cap) {
    for (size_t i = 0; i < m; i++) {
      shard[i] = p[i].from;
      dot[i] = p[i].dot;
    }
    g->req_shard.len = g->req_dot.len = 0;
  }
  free(p);
  return m;
}

/* request_replies()  mod.rs:152-157: sizes, then taken in list order:
 * to[nr], kind[nr] (0 Info, 1 Executed), dot[nr], cmask[nr] (Info: the
 * command's shards), doff[nr+1] into ddot / dmask (Info: the vertex's deps) */
void fo_graph_replies_size(const fo_graph *g, size_t *nr, size_t *nd) {
  *nr = g->rep_dot.len;
  *nd = g->rep_ddot.len;
}
void fo_graph_replies_take(fo_graph *g, uint64_t *to, uint64_t *kind, uint64_t *dot,
                           uint64_t *cmask, uint64_t *doff, uint64_t *ddot, uint64_t *dmask) {
  size_t nr = g->rep_dot.len, nd = g->rep_ddot.len;
  memcpy(to, g->rep_to.a, nr * sizeof(uint64_t));
  memcpy(kind, g->rep_kind.a, nr * sizeof(uint64_t));
  memcpy(dot, g->rep_dot.a, nr * sizeof(uint64_t));
  memcpy(cmask, g->rep_cmask.a, nr * sizeof(uint64_t));
  doff[0] = 0;
  memcpy(doff + 1, g->rep_doff.a, nr * sizeof(uint64_t));
  if (nd) {
    memcpy(ddot, g->rep_ddot.a, nd * sizeof(uint64_t));
    memcpy(dmask, g->rep_dmask.a, nd * sizeof(uint64_t));
  }
  g->rep_to.len = g->rep_kind.len = g->rep_dot.len = g->rep_cmask.len = g->rep_doff.len = 0;
  g->rep_ddot.len = g->rep_dmask.len = 0;
}

/* handle_request_reply's Executed{dot}  mod.rs:393-405: the executed clock
 * advances and the dot's pending children are retried */
size_t fo_graph_mark_executed(fo_graph *g, uint64_t dot) {
  ae_add(&g->executed, dot);
  vec64 dots = {0};
  vpush(&dots, dot);
  size_t total = 0;
  check_pending(g, &dots, &total);
  free(dots.a);
  return total;
}

int fo_graph_violation(const fo_graph *g) { return g->violation; }

void fo_graph_index_only(fo_graph *g, uint64_t dot, const uint64_t *keys,
                         size_t nkeys, const uint64_t *deps, size_t ndeps) {
  index_vertex(g, dot, keys, nkeys, deps, ndeps, 0, NULL);
}

void fo_graph_set_executed_frontier(fo_graph *g, uint32_t source,
                                    uint64_t seq) {
  g->executed.frontier[source & 255] = seq;
}

int fo_graph_find_scc(fo_graph *g, int first_find, uint64_t dot,
                      size_t *ready, size_t *nfound, uint64_t *missing,
                      size_t missing_cap, size_t *nmissing) {
  finder_info fi;
  size_t total = 0;
  find_scc(g, first_find, dot, &total, &fi);
  *ready = total;
  *nfound = fi.dots.len;
  *nmissing = emit(fi.missing.a, fi.missing.len, missing, missing_cap);
  int kind = fi.kind == FR_FOUND ? 0 : (fi.kind == FR_MISSING ? 1 : 2);
  fi_free(&fi);
  return kind;
}

int fo_graph_executed(const fo_graph *g, uint64_t dot) {
  return ae_contains(&g->executed, dot);
}

size_t fo_graph_drain(fo_graph *g, uint64_t *dots, uint64_t *scc_label,
                      size_t cap) {
  size_t c = 0;
  while (g->qhead < g->qtail && c < cap) {
    if (dots) dots[c] = g->q[g->qhead].dot;
    if (scc_label) scc_label[c] = g->q[g->qhead].label;
    g->qhead++;
    c++;
  }
  return c;
}

size_t fo_graph_pending_count(const fo_graph *g) { return g->vindex.len; }

size_t fo_graph_run(uint32_t process_id, uint32_t n, uint32_t f, size_t ncmd,
                    const uint64_t *dot, const uint32_t *key_off,
                    const uint64_t *keys, const uint32_t *dep_off,
                    const uint64_t *deps, uint64_t *exec_dot,
                    uint64_t *scc_label, uint64_t key_space,
                    uint32_t *key_seq_off, uint64_t *key_seq) {
  fo_graph *g = fo_graph_new(process_id, 0, n, f, 1);
  u64map where; /* dot -> command index (to find keys of executed dots) */
  map_init(&where, ncmd);
  for (size_t i = 0; i < ncmd; i++) map_put(&where, dot[i], i);
  size_t executed = 0;
  for (size_t i = 0; i < ncmd; i++) {
    fo_graph_add(g, dot[i], keys + key_off[i], key_off[i + 1] - key_off[i],
                 deps + dep_off[i], dep_off[i + 1] - dep_off[i]);
    executed += fo_graph_drain(g, exec_dot + executed, scc_label + executed,
                               ncmd - executed);
  }
  /* ExecutionOrderMonitor (monitor.rs:20-28), dense key ids */
  if (key_seq_off && key_seq) {
    memset(key_seq_off, 0, (key_space + 1) * sizeof(uint32_t));
    for (size_t e = 0; e < executed; e++) {
      size_t i = (size_t)*map_get(&where, exec_dot[e]);
      for (uint32_t t = key_off[i]; t < key_off[i + 1]; t++)
        key_seq_off[keys[t] + 1]++;
    }
    for (uint64_t k = 0; k < key_space; k++)
      key_seq_off[k + 1] += key_seq_off[k];
    uint32_t *fill = (uint32_t *)xmalloc(key_space * sizeof(uint32_t));
    memcpy(fill, key_seq_off, key_space * sizeof(uint32_t));
    for (size_t e = 0; e < executed; e++) {
      size_t i = (size_t)*map_get(&where, exec_dot[e]);
      for (uint32_t t = key_off[i]; t < key_off[i + 1]; t++)
        key_seq[fill[keys[t]]++] = exec_dot[e];
    }
    free(fill);
  }
  map_free(&where);
  fo_graph_free(g);
  return executed;
}

/* ------------------------------------------------------------------ */
/* PredecessorsGraph -- Caesar's executor                               */
/* (fantoch_ps/src/executor/pred/mod.rs:26-352, index.rs)               */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t dot, clock; /* clock packed (seq << 8) | process_id: Clock's Ord */
  uint64_t deps_at;
  uint32_t ndeps;
  uint32_t missing; /* Vertex::missing_deps (index.rs) */
} pvertex;

struct fo_pred {
  aeclock committed, executed; /* mod.rs:29-30 */
  pvertex *v;
  size_t nv, vcap;
  u64map index;       /* VertexIndex: dot -> slot + 1 */
  vec64 deps;         /* dep pool */
  u64map p1, p2;      /* PendingIndex (phase one / two): dep -> head + 1 */
  pend_node *pn;      /* linked lists of waiting dots */
  size_t npn, pncap;
  vec64 to_execute;   /* mod.rs:37 */
  vec64 stack;        /* save_to_execute cascade (explicit stack) */
};

fo_pred *fo_pred_new(uint32_t process_id) {
  fo_pred *p = (fo_pred *)calloc(1, sizeof(fo_pred));
  ae_init(&p->committed);
  ae_init(&p->executed);
  map_init(&p->index, 1024);
  map_init(&p->p1, 256);
  map_init(&p->p2, 256);
  (void)process_id;
  return p;
}

void fo_pred_free(fo_pred *p) {
  map_free(&p->committed.exc);
  map_free(&p->executed.exc);
  map_free(&p->index);
  map_free(&p->p1);
  map_free(&p->p2);
  free(p->v);
  free(p->deps.a);
  free(p->pn);
  free(p->to_execute.a);
  free(p->stack.a);
  free(p);
}

static pvertex *pred_find(fo_pred *p, uint64_t dot) {
  uint64_t *s = map_get(&p->index, dot);
  return s ? &p->v[*s - 1] : NULL;
}

/* PendingIndex::index(dot, dep): dot waits on dep (insertion order kept) */
static void pend_index(fo_pred *p, u64map *m, uint64_t dot, uint64_t dep) {
  if (p->npn == p->pncap) {
    p->pncap = p->pncap ? p->pncap * 2 : 256;
    p->pn = (pend_node *)xrealloc(p->pn, p->pncap * sizeof(pend_node));
  }
  uint64_t *h = map_get(m, dep);
  /* append at the tail: walk (lists are short) */
  pend_node nd = {dot, -1};
  p->pn[p->npn] = nd;
  if (!h) {
    map_put(m, dep, (uint64_t)p->npn + 1);
  } else {
    int64_t i = (int64_t)(*h - 1);
    while (p->pn[i].next >= 0) i = p->pn[i].next;
    p->pn[i].next = (int64_t)p->npn;
  }
  p->npn++;
}

/* PendingIndex::remove(dep) -> waiting dots, into out (insertion order) */
static void pend_remove(fo_pred *p, u64map *m, uint64_t dep, vec64 *out) {
  uint64_t head;
  if (!map_del(m, dep, &head)) return;
  for (int64_t i = (int64_t)(head - 1); i >= 0; i = p->pn[i].next) vpush(out, p->pn[i].child);
}

static void pred_save_to_execute(fo_pred *p, uint64_t dot);

/* move_to_phase_two (mod.rs:186-253) */
static void pred_phase_two(fo_pred *p, uint64_t dot) {
  pvertex *v = pred_find(p, dot);
  uint32_t count = 0;
  for (uint32_t e = 0; e < v->ndeps; e++) {
    uint64_t d = p->deps.a[v->deps_at + e];
    if (ae_contains(&p->executed, d)) continue;
    pvertex *dv = pred_find(p, d);
    if (!dv) {
      fprintf(stderr, "oracle: non-executed dependency must exist\n");
      abort();
    }
    if (dv->clock < v->clock) { /* only deps with a lower clock (:224) */
      count++;
      pend_index(p, &p->p2, dot, d);
    }
  }
  if (count) v->missing = count;
  else pred_save_to_execute(p, dot);
}

/* move_to_phase_one (mod.rs:132-182) */
static void pred_phase_one(fo_pred *p, uint64_t dot) {
  pvertex *v = pred_find(p, dot);
  uint32_t count = 0;
  for (uint32_t e = 0; e < v->ndeps; e++) {
    uint64_t d = p->deps.a[v->deps_at + e];
    if (!ae_contains(&p->committed, d)) {
      count++;
      pend_index(p, &p->p1, dot, d);
    }
  }
  if (count) v->missing = count;
  else pred_phase_two(p, dot);
}

/* save_to_execute (mod.rs:322-351) and the try_phase_two_pending cascade
 * (:299-320), depth first like the reference's recursion, on an explicit
 * stack */
static void pred_save_to_execute(fo_pred *p, uint64_t dot) {
  size_t base = p->stack.len;
  vpush(&p->stack, dot);
  vec64 kids = {0};
  while (p->stack.len > base) {
    uint64_t d = p->stack.a[--p->stack.len];
    if (ae_contains(&p->executed, d)) {
      fprintf(stderr, "oracle: command executed twice\n");
      abort();
    }
    ae_add(&p->executed, d);
    uint64_t slot;
    map_del(&p->index, d, &slot);
    vpush(&p->to_execute, d);
    kids.len = 0;
    pend_remove(p, &p->p2, d, &kids);
    /* children that become ready, pushed in reverse so the first runs first */
    size_t mark = p->stack.len;
    for (size_t i = 0; i < kids.len; i++) {
      pvertex *c = pred_find(p, kids.a[i]);
      if (--c->missing == 0) vpush(&p->stack, kids.a[i]);
    }
    if (p->stack.len > mark + 1) {
      for (size_t i = mark, j = p->stack.len - 1; i < j; i++, j--) {
        uint64_t t = p->stack.a[i];
        p->stack.a[i] = p->stack.a[j];
        p->stack.a[j] = t;
      }
    }
  }
  free(kids.a);
}

size_t fo_pred_add(fo_pred *p, uint64_t dot, uint64_t clock, const uint64_t *deps,
                   size_t ndeps) {
  size_t before = p->to_execute.len;
  /* deps.remove(&dot) (mod.rs:106-109); HashSet: no duplicates */
  size_t at = p->deps.len;
  for (size_t i = 0; i < ndeps; i++)
    if (deps[i] != dot) vpush(&p->deps, deps[i]);
  size_t nd = sort_unique(p->deps.a + at, p->deps.len - at);
  p->deps.len = at + nd;
  /* index_committed_command (mod.rs:255-274) */
  if (ae_contains(&p->committed, dot)) {
    fprintf(stderr, "oracle: dot committed twice\n");
    abort();
  }
  ae_add(&p->committed, dot);
  if (p->nv == p->vcap) {
    p->vcap = p->vcap ? p->vcap * 2 : 1024;
    p->v = (pvertex *)xrealloc(p->v, p->vcap * sizeof(pvertex));
  }
  pvertex nv = {dot, clock, at, (uint32_t)nd, 0};
  p->v[p->nv] = nv;
  map_put(&p->index, dot, (uint64_t)p->nv + 1);
  p->nv++;
  /* try_phase_one_pending (mod.rs:276-297) */
  vec64 w = {0};
  pend_remove(p, &p->p1, dot, &w);
  for (size_t i = 0; i < w.len; i++) {
    pvertex *c = pred_find(p, w.a[i]);
    if (--c->missing == 0) pred_phase_two(p, w.a[i]);
  }
  free(w.a);
  /* move_to_phase_one (mod.rs:118) */
  pred_phase_one(p, dot);
  return p->to_execute.len - before;
}

size_t fo_pred_drain(fo_pred *p, uint64_t *dots, size_t cap) {
  size_t n = p->to_execute.len < cap ? p->to_execute.len : cap;
  if (dots) memcpy(dots, p->to_execute.a, n * sizeof(uint64_t));
  memmove(p->to_execute.a, p->to_execute.a + n, (p->to_execute.len - n) * sizeof(uint64_t));
  p->to_execute.len -= n;
  return n;
}

size_t fo_pred_pending_count(const fo_pred *p) { return p->index.len; }
