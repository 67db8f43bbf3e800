/*
 * bine_oracle.c -- CPU restatement of libbine's reduce-family.
 *
 * TEST INFRASTRUCTURE ONLY (see bine_oracle.h).  Never linked into the product.
 *
 * Every function below names the reference lines it restates.  All P ranks are
 * simulated in one process; a "superstep" is one round of matching
 * point-to-point calls (MPI_Sendrecv, or a batch of Isend/Irecv + Wait) after
 * which each rank does its local work.  Messages are copied when posted, so a
 * superstep behaves exactly like the blocking MPI calls it stands for.
 */
#define _GNU_SOURCE
#include "bine_oracle.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EL(p, i) ((char *)(p) + (size_t)(i) * esz)

/* ----------------------------------------------------------------------- */
/* element types and MPI_Reduce_local                                       */
/* ----------------------------------------------------------------------- */

size_t orc_dtype_size(int dt) {
  switch (dt) {
    case ORC_INT8: case ORC_UINT8: return 1;
    case ORC_INT16: case ORC_UINT16: return 2;
    case ORC_INT32: case ORC_UINT32: case ORC_FLOAT: return 4;
    case ORC_INT64: case ORC_UINT64: case ORC_DOUBLE: return 8;
    case ORC_FLOAT_INT: case ORC_2INT: case ORC_SHORT_INT: return 8;
    case ORC_DOUBLE_INT: case ORC_LONG_INT: return 16;
    case ORC_C_FLOAT_COMPLEX: return 8;
    case ORC_C_DOUBLE_COMPLEX: return 16;
    default: return 0;
  }
}

/* MPICH 3.3.2 MPIR_OP_TYPE_REDUCE_CASE: a = inout, b = in, a[i] = OP(a[i], b[i])
 * with MPIR_MAX(a,b) = a > b ? a : b and MPIR_MIN(a,b) = a < b ? a : b.
 * Signed integer SUM/PROD wrap (computed unsigned: same bits, no UB).
 * Logical ops (opland.c / oplor.c / oplxor.c): MPIR_LLAND(a,b) = a && b,
 * MPIR_LLOR = a || b, MPIR_LLXOR = (a && !b) || (!a && b) -- C truthiness, the
 * 0/1 result stored in the element type; MPICH accepts them on floating types
 * too.  Bitwise ops (opband.c / opbor.c / opbxor.c): integer types only
 * (floating types: MPI_ERR_OP, here -1).  Checked against MPICH's own
 * MPI_Reduce_local by tests/golden (the reference's vectors, sparse inputs). */
#define RL_LOGIC                                                              \
      case ORC_LAND: for (size_t i = 0; i < n; i++) a[i] = (a[i] && b[i]); break; \
      case ORC_LOR:  for (size_t i = 0; i < n; i++) a[i] = (a[i] || b[i]); break; \
      case ORC_LXOR: for (size_t i = 0; i < n; i++) a[i] = ((a[i] && !b[i]) || (!a[i] && b[i])); break

#define RL_INT(T, UT)                                                         \
  do {                                                                        \
    T *a = (T *)inout; const T *b = (const T *)in;                            \
    switch (op) {                                                             \
      case ORC_SUM:  for (size_t i = 0; i < n; i++) a[i] = (T)((UT)a[i] + (UT)b[i]); break; \
      case ORC_PROD: for (size_t i = 0; i < n; i++) a[i] = (T)((UT)a[i] * (UT)b[i]); break; \
      case ORC_MAX:  for (size_t i = 0; i < n; i++) a[i] = a[i] > b[i] ? a[i] : b[i]; break; \
      case ORC_MIN:  for (size_t i = 0; i < n; i++) a[i] = a[i] < b[i] ? a[i] : b[i]; break; \
      case ORC_BAND: for (size_t i = 0; i < n; i++) a[i] = (T)(a[i] & b[i]); break; \
      case ORC_BOR:  for (size_t i = 0; i < n; i++) a[i] = (T)(a[i] | b[i]); break; \
      case ORC_BXOR: for (size_t i = 0; i < n; i++) a[i] = (T)(a[i] ^ b[i]); break; \
      RL_LOGIC;                                                               \
      default: return -1;                                                     \
    }                                                                         \
  } while (0)

#define RL_FLT(T)                                                             \
  do {                                                                        \
    T *a = (T *)inout; const T *b = (const T *)in;                            \
    switch (op) {                                                             \
      case ORC_SUM:  for (size_t i = 0; i < n; i++) a[i] = a[i] + b[i]; break; \
      case ORC_PROD: for (size_t i = 0; i < n; i++) a[i] = a[i] * b[i]; break; \
      case ORC_MAX:  for (size_t i = 0; i < n; i++) a[i] = a[i] > b[i] ? a[i] : b[i]; break; \
      case ORC_MIN:  for (size_t i = 0; i < n; i++) a[i] = a[i] < b[i] ? a[i] : b[i]; break; \
      RL_LOGIC;                                                               \
      default: return -1;                                                     \
    }                                                                         \
  } while (0)

/* MPI's pair types, C layout, with the padding spelled out as members: C
 * leaves implicit padding unspecified, and gcc -O2 does store garbage there
 * when it merges the field updates (measured); as members, the inout
 * operand's padding bytes survive, as on the device */
typedef struct { float v; int i; } orc_float_int;
typedef struct { double v; int i, pad_; } orc_double_int;
typedef struct { long v; int i, pad_; } orc_long_int;
typedef struct { int v; int i; } orc_2int;
typedef struct { short v, pad_; int i; } orc_short_int;

/* MPICH 3.3.2 opmaxloc.c / opminloc.c, a = inout, b = in: equal values keep
 * MPL_MIN of the indices, a strictly larger (MAXLOC) / smaller (MINLOC) `in`
 * value replaces the pair.  Field by field (MPICH assigns the struct; its
 * padding bytes are not part of the type map and never travel). */
#define RL_PAIR(T)                                                            \
  do {                                                                        \
    T *a = (T *)inout; const T *b = (const T *)in;                            \
    if (op != ORC_MAXLOC && op != ORC_MINLOC) return -1;                      \
    for (size_t i = 0; i < n; i++) {                                          \
      if (a[i].v == b[i].v) a[i].i = a[i].i < b[i].i ? a[i].i : b[i].i;       \
      else if (op == ORC_MAXLOC ? a[i].v < b[i].v : a[i].v > b[i].v) {        \
        a[i].v = b[i].v;                                                      \
        a[i].i = b[i].i;                                                      \
      }                                                                       \
    }                                                                         \
  } while (0)

/* MPICH 3.3.2 opsum.c / opprod.c on the C complex types: MPIR_LSUM /
 * MPIR_LPROD on float _Complex / double _Complex, a = inout, b = in.  For
 * finite operands gcc's complex product is (a.re b.re - a.im b.im) +
 * (a.re b.im + a.im b.re) i, no FMA on x86-64; its Annex G NaN recovery
 * (__mulsc3, both parts NaN) is not restated -- the vectors use finite values */
typedef struct { float re, im; } orc_cfloat;
typedef struct { double re, im; } orc_cdouble;
#define RL_CPLX(T, V)                                                         \
  do {                                                                        \
    T *a = (T *)inout; const T *b = (const T *)in;                            \
    switch (op) {                                                             \
      case ORC_SUM:                                                           \
        for (size_t i = 0; i < n; i++) { a[i].re = a[i].re + b[i].re; a[i].im = a[i].im + b[i].im; } \
        break;                                                                \
      case ORC_PROD:                                                          \
        for (size_t i = 0; i < n; i++) {                                      \
          const V re = a[i].re * b[i].re - a[i].im * b[i].im;                 \
          const V im = a[i].re * b[i].im + a[i].im * b[i].re;                 \
          a[i].re = re;                                                       \
          a[i].im = im;                                                       \
        }                                                                     \
        break;                                                                \
      default: return -1;                                                     \
    }                                                                         \
  } while (0)

int orc_reduce_local(const void *in, void *inout, size_t n, int dtype, int op) {
  if (dtype < ORC_FLOAT_INT && (op == ORC_MAXLOC || op == ORC_MINLOC)) return -1;
  switch (dtype) {
    case ORC_C_FLOAT_COMPLEX:  RL_CPLX(orc_cfloat, float); break;
    case ORC_C_DOUBLE_COMPLEX: RL_CPLX(orc_cdouble, double); break;
    case ORC_FLOAT_INT:  RL_PAIR(orc_float_int); break;
    case ORC_DOUBLE_INT: RL_PAIR(orc_double_int); break;
    case ORC_LONG_INT:   RL_PAIR(orc_long_int); break;
    case ORC_2INT:       RL_PAIR(orc_2int); break;
    case ORC_SHORT_INT:  RL_PAIR(orc_short_int); break;
    case ORC_INT8:   RL_INT(int8_t, uint8_t); break;
    case ORC_UINT8:  RL_INT(uint8_t, uint8_t); break;
    case ORC_INT16:  RL_INT(int16_t, uint16_t); break;
    case ORC_UINT16: RL_INT(uint16_t, uint16_t); break;
    case ORC_INT32:  RL_INT(int32_t, uint32_t); break;
    case ORC_UINT32: RL_INT(uint32_t, uint32_t); break;
    case ORC_INT64:  RL_INT(int64_t, uint64_t); break;
    case ORC_UINT64: RL_INT(uint64_t, uint64_t); break;
    case ORC_FLOAT:  RL_FLT(float); break;
    case ORC_DOUBLE: RL_FLT(double); break;
    default: return -1;
  }
  return 0;
}

/* pico_core_utils.c:902-923 (rand_r distributions).  The int64 pair is drawn
 * high word first. */
/* pico_core has no generator for MPI's pair types; the golden harness
 * (oracle/ref_golden.c fill) and this one draw value = rand_r() % 16 (halved
 * for the floating values: ties and fractions) and index = rand_r() % 1000,
 * padding 0 */
#define FILL_PAIR(T, VT, HALF)                                                \
  do {                                                                        \
    T *p = (T *)buf;                                                          \
    memset(p, 0, n * sizeof(T));                                              \
    for (size_t i = 0; i < n; i++) {                                          \
      const int r = rand_r(&seed) % 16;                                       \
      p[i].v = HALF ? (VT)r / (VT)2 : (VT)r;                                  \
      p[i].i = rand_r(&seed) % 1000;                                          \
    }                                                                         \
    return 0;                                                                 \
  } while (0)

int orc_fill(void *buf, int dtype, size_t n, unsigned int seed) {
  switch (dtype) {
    case ORC_FLOAT_INT:  FILL_PAIR(orc_float_int, float, 1);
    case ORC_DOUBLE_INT: FILL_PAIR(orc_double_int, double, 1);
    case ORC_LONG_INT:   FILL_PAIR(orc_long_int, long, 0);
    case ORC_2INT:       FILL_PAIR(orc_2int, int, 0);
    case ORC_SHORT_INT:  FILL_PAIR(orc_short_int, short, 0);
    case ORC_C_FLOAT_COMPLEX:   /* pico_core's fp distribution, re then im */
      for (size_t i = 0; i < 2 * n; i++) ((float *)buf)[i] = (float)rand_r(&seed) / (float)RAND_MAX * 100.0f;
      return 0;
    case ORC_C_DOUBLE_COMPLEX:
      for (size_t i = 0; i < 2 * n; i++) ((double *)buf)[i] = (double)rand_r(&seed) / (double)RAND_MAX * 100.0;
      return 0;
    default: break;
  }
  for (size_t i = 0; i < n; i++) {
    switch (dtype) {
      case ORC_INT8:   ((int8_t *)buf)[i] = (int8_t)((rand_r(&seed) % 256) - 128); break;
      case ORC_INT16:  ((int16_t *)buf)[i] = (int16_t)((rand_r(&seed) % 65536) - 32768); break;
      case ORC_INT32:  ((int32_t *)buf)[i] = (int32_t)rand_r(&seed); break;
      case ORC_INT64: {
        int64_t hi = (int64_t)rand_r(&seed) << 32;
        ((int64_t *)buf)[i] = hi | rand_r(&seed);
        break;
      }
      case ORC_FLOAT:  ((float *)buf)[i] = (float)rand_r(&seed) / (float)RAND_MAX * 100.0f; break;
      case ORC_DOUBLE: ((double *)buf)[i] = (double)rand_r(&seed) / (double)RAND_MAX * 100.0; break;
      case ORC_UINT8:  ((uint8_t *)buf)[i] = (uint8_t)(rand_r(&seed) % 256); break;
      case ORC_UINT16: ((uint16_t *)buf)[i] = (uint16_t)(rand_r(&seed) % 65536); break;
      case ORC_UINT32: ((uint32_t *)buf)[i] = (uint32_t)rand_r(&seed); break;
      case ORC_UINT64: {
        uint64_t hi = (uint64_t)rand_r(&seed) << 32;
        ((uint64_t *)buf)[i] = hi | (uint64_t)rand_r(&seed);
        break;
      }
      default: return -1;
    }
  }
  return 0;
}

/* ----------------------------------------------------------------------- */
/* schedule math -- libbine_utils.h                                          */
/* ----------------------------------------------------------------------- */

/* rhos[] (libbine_utils.h:44-45): rho_s = sum_{i<=s} (-2)^i */
static int rho(int step) {
  int v = 0, p = 1;
  for (int i = 0; i <= step; i++) { v += p; p *= -2; }
  return v;
}

/* pi(), libbine_utils.h:129-138 */
int orc_pi(int rank, int step, int P) {
  int d = (rank & 1) == 0 ? (rank + rho(step)) % P : (rank - rho(step)) % P;
  if (d < 0) d += P;
  return d;
}

static int is_pow2(int v) { return (v & (v - 1)) == 0; }        /* :267-269 */
static int log_2(int v) {                                           /* :279-288 */
  if (v < 1) return -1;
  int l = 31 - __builtin_clz((unsigned)v);
  if (!is_pow2(v)) l++;
  return l;
}
static int next_pow2(int v) {                                       /* :298-309 */
  if (v < 0) return -1;
  if (v == 0) return 1;
  return (int)(1u << (32 - __builtin_clz((unsigned)v)));
}
static int hibit(int value, int start) {                            /* :327-341 */
  unsigned mask = (unsigned)value & ((1u << start) - 1u);
  if (!mask) return -1;
  return 31 - __builtin_clz(mask);
}
static uint32_t b2nb(int32_t bin) {                                 /* :509-513 */
  if (bin > 0x55555555) return UINT32_MAX;
  const uint32_t m = 0xAAAAAAAAu;
  return (m + (uint32_t)bin) ^ m;
}
static int32_t nb2b(uint32_t neg) {                                 /* :515-518 */
  const uint32_t m = 0xAAAAAAAAu;
  return (int32_t)((m ^ neg) - m);
}
static int mod(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }  /* :520-523 */
/* smallest_/largest_negabinary[] (:47-50): the most negative / positive value
 * representable with n negabinary digits */
static int nb_lo(int n) { int v = 0; for (int i = 1; i < n; i += 2) v -= 1 << i; return v; }
static int nb_hi(int n) { int v = 0; for (int i = 0; i < n; i += 2) v += 1 << i; return v; }
static int in_range(int x, int n) { return x >= nb_lo(n) && x <= nb_hi(n); }   /* :524-526 */
static uint32_t rev32(uint32_t x) {                                 /* :528-535 */
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0f0f0f0fu) | ((x & 0x0f0f0f0fu) << 4);
  x = ((x >> 8) & 0x00ff00ffu) | ((x & 0x00ff00ffu) << 8);
  return (x >> 16) | (x << 16);
}
static uint32_t shr(uint32_t x, int s) { return s >= 32 ? 0 : x >> s; }

/* get_rank_negabinary_representation(), :537-570 -- including the decimal
 * literal 80000000 of the tie-break at :564. */
static uint32_t nb_repr(uint32_t P, uint32_t rank, int *bad) {
  uint32_t nba = UINT32_MAX, nbb = UINT32_MAX;
  int nbits = log_2((int)P);
  if (rank % 2) {
    if (in_range((int)rank, nbits)) nba = b2nb((int32_t)rank);
    if (in_range((int)rank - (int)P, nbits)) nbb = b2nb((int32_t)rank - (int32_t)P);
  } else {
    if (in_range(-(int)rank, nbits)) nba = b2nb(-(int32_t)rank);
    if (in_range(-(int)rank + (int)P, nbits)) nbb = b2nb(-(int32_t)rank + (int32_t)P);
  }
  if (nba == UINT32_MAX && nbb == UINT32_MAX) { if (bad) *bad = 1; return 0; }
  if (nba == UINT32_MAX) return nbb;
  if (nbb == UINT32_MAX) return nba;
  int sh = 32 - nbits;
  uint32_t msb = (uint32_t)(sh < 32 ? (80000000 >> sh) : 80000000);
  return (nba & msb) ? nba : nbb;
}

/* remap_rank(), :572-578 */
uint32_t orc_remap_rank(uint32_t P, uint32_t rank) {
  uint32_t v = nb_repr(P, rank, NULL);
  v ^= v >> 1;
  return shr(rev32(v), 32 - log_2((int)P));
}

/* get_nu() / nb_to_nu(), :611-648 */
static uint32_t nb_to_nu(uint32_t nb, uint32_t size) {
  return shr(rev32(nb ^ (nb >> 1)), 32 - log_2((int)size));
}
uint32_t orc_get_nu(uint32_t rank, uint32_t size) {
  uint32_t nba = UINT32_MAX, nbb = UINT32_MAX;
  int nbits = log_2((int)size);
  if (rank % 2) {
    if (in_range((int)rank, nbits)) nba = b2nb((int32_t)rank);
    if (in_range((int)rank - (int)size, nbits)) nbb = b2nb((int32_t)rank - (int32_t)size);
  } else {
    if (in_range(-(int)rank, nbits)) nba = b2nb(-(int32_t)rank);
    if (in_range(-(int)rank + (int)size, nbits)) nbb = b2nb(-(int32_t)rank + (int32_t)size);
  }
  if (nba == UINT32_MAX && nbb == UINT32_MAX) return 0;
  if (nba == UINT32_MAX) return nb_to_nu(nbb, size);
  if (nbb == UINT32_MAX) return nb_to_nu(nba, size);
  int a = (int)nb_to_nu(nba, size), b = (int)nb_to_nu(nbb, size);
  return (uint32_t)(a < b ? a : b);
}

static uint32_t inverse_rank(uint32_t P, uint32_t rank) {           /* :580-583 */
  return shr(rev32(rank), 32 - log_2((int)P));
}
static uint32_t mirror_perm(uint32_t x, int nbits) {                 /* :418-426 */
  return shr(rev32(x), 32 - nbits);
}

/* Static tables (libbine_utils_bitmaps.c:10-56).  The reference ships them as
 * literals; here they are regenerated.  Rule (checked against every table for
 * P = 2..256 in tests/test_oracle.py): the static final-block permutation is the
 * remap permutation with each last-step pair {r, pi(r, n-1)} -- the two ranks
 * sharing blocks 2k, 2k+1 -- put in ascending rank order:
 *   perm[r] = (remap_rank(P, r) & ~1) | (r > pi(r, n-1, P)).
 * A rank's window at step s is the aligned run of P >> (s+1) blocks holding
 * perm[r]: recv[r][s] = perm[r] & ~(w - 1); send[r][s] = recv[pi(r,s)][s]. */
int orc_static_tables(int P, int *perm, int *send_tab, int *recv_tab) {
  if (P < 2 || !is_pow2(P)) return -1;
  int n = log_2(P);
  for (int r = 0; r < P; r++)
    perm[r] = (int)(orc_remap_rank((uint32_t)P, (uint32_t)r) & ~1u) | (r > orc_pi(r, n - 1, P) ? 1 : 0);
  for (int r = 0; r < P; r++)
    for (int s = 0; s < n; s++) {
      int w = P >> (s + 1);
      recv_tab[r * n + s] = perm[r] & ~(w - 1);
    }
  for (int r = 0; r < P; r++)
    for (int s = 0; s < n; s++) send_tab[r * n + s] = recv_tab[orc_pi(r, s, P) * n + s];
  return 0;
}

/* ----------------------------------------------------------------------- */
/* point-to-point superstep simulator                                        */
/* ----------------------------------------------------------------------- */

#define ANY_SRC (-7)

typedef struct { int src, dst, tag; size_t bytes; char *data; int used; } msg_t;
typedef struct { int src, dst, tag; char *ptr; size_t cap; } rcv_t;
typedef struct {
  msg_t *m; int nm, cm;
  rcv_t *r; int nr, cr;
} board_t;

static void b_send_t(board_t *b, int src, int dst, const void *p, size_t bytes, int tag) {
  if (dst < 0) return;                       /* MPI_PROC_NULL */
  if (b->nm == b->cm) { b->cm = b->cm ? 2 * b->cm : 16; b->m = (msg_t *)realloc(b->m, sizeof(msg_t) * (size_t)b->cm); }
  msg_t *x = &b->m[b->nm++];
  x->src = src; x->dst = dst; x->tag = tag; x->bytes = bytes; x->used = 0;
  x->data = (char *)malloc(bytes ? bytes : 1);
  if (bytes) memcpy(x->data, p, bytes);
}

static void b_recv_t(board_t *b, int dst, int src, void *p, size_t cap, int tag) {
  if (src == -1) return;                     /* MPI_PROC_NULL */
  if (b->nr == b->cr) { b->cr = b->cr ? 2 * b->cr : 16; b->r = (rcv_t *)realloc(b->r, sizeof(rcv_t) * (size_t)b->cr); }
  rcv_t *x = &b->r[b->nr++];
  x->src = src; x->dst = dst; x->tag = tag; x->ptr = (char *)p; x->cap = cap;
}

static void b_send(board_t *b, int src, int dst, const void *p, size_t bytes) { b_send_t(b, src, dst, p, bytes, 0); }
static void b_recv(board_t *b, int dst, int src, void *p, size_t cap) { b_recv_t(b, dst, src, p, cap, 0); }

/* Deliver every posted receive (per-pair, per-tag FIFO: MPI's non-overtaking
 * rule).  Truncation marks the receiving rank's return code; an unmatched send
 * or receive means the reference would block forever. */
static int b_deliver(board_t *b, int *rets) {
  int status = 0;
  for (int i = 0; i < b->nr; i++) {
    rcv_t *r = &b->r[i];
    msg_t *hit = NULL;
    for (int j = 0; j < b->nm; j++) {
      msg_t *m = &b->m[j];
      if (!m->used && m->dst == r->dst && m->tag == r->tag && (r->src == ANY_SRC || m->src == r->src)) { hit = m; break; }
    }
    if (!hit) { status = ORC_DEADLOCK; continue; }
    hit->used = 1;
    size_t nb = hit->bytes;
    if (nb > r->cap) { nb = r->cap; if (rets && rets[r->dst] == 0) rets[r->dst] = ORC_ERR_TRUNCATE; }
    if (nb) memcpy(r->ptr, hit->data, nb);
  }
  for (int j = 0; j < b->nm; j++) {
    if (!b->m[j].used) status = ORC_DEADLOCK;
    free(b->m[j].data);
  }
  b->nm = 0; b->nr = 0;
  return status;
}

static void b_free(board_t *b) { free(b->m); free(b->r); memset(b, 0, sizeof *b); }

typedef struct {
  int P, dtype, op;
  size_t esz;
  board_t b;
  int dead;
} ctx_t;

static void deliver(ctx_t *c, int *rets) {
  int s = b_deliver(&c->b, rets);
  if (s) c->dead = s;
}
static void red(ctx_t *c, const void *in, void *inout, size_t n) {
  if (n) orc_reduce_local(in, inout, n, c->dtype, c->op);
}

static char **alloc_ranks(int P, size_t bytes) {
  char **v = (char **)malloc(sizeof(char *) * (size_t)P);
  for (int r = 0; r < P; r++) v[r] = (char *)calloc(bytes ? bytes : 1, 1);
  return v;
}
static void free_ranks(char **v, int P) { for (int r = 0; r < P; r++) free(v[r]); free(v); }

/* ----------------------------------------------------------------------- */
/* allreduce -- libbine_allreduce.c                                          */
/* ----------------------------------------------------------------------- */

/* allreduce_recursivedoubling, :17-135 */
static void ar_recursivedoubling(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  if (P == 1) { if (nb) memcpy(R[0], S[0], nb); return; }
  char **inpl = alloc_ranks(P, nb);
  char **tsend = (char **)malloc(sizeof(char *) * (size_t)P);
  int *newrank = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) { if (nb) memcpy(inpl[r], S[r], nb); tsend[r] = inpl[r]; }
  int adj = next_pow2(P) >> 1, extra = P - adj;
  for (int r = 0; r < P; r++) {                                      /* :66-82 */
    if (r < 2 * extra) {
      if (r % 2 == 0) { b_send(&c->b, r, r + 1, tsend[r], nb); newrank[r] = -1; }
      else { b_recv(&c->b, r, r - 1, R[r], nb); newrank[r] = r >> 1; }
    } else newrank[r] = r - extra;
  }
  deliver(c, rets);
  for (int r = 0; r < 2 * extra; r += 2) red(c, R[r + 1], tsend[r + 1], count);
  for (int dist = 1; dist < adj; dist <<= 1) {                       /* :89-103 */
    for (int r = 0; r < P; r++) {
      if (newrank[r] < 0) continue;
      int nrem = newrank[r] ^ dist;
      int remote = nrem < extra ? nrem * 2 + 1 : nrem + extra;
      b_send(&c->b, r, remote, tsend[r], nb);
      b_recv(&c->b, r, remote, R[r], nb);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) if (newrank[r] >= 0) red(c, R[r], tsend[r], count);
  }
  for (int r = 0; r < 2 * extra; r++) {                              /* :110-119 */
    if (r % 2 == 0) { b_recv(&c->b, r, r + 1, R[r], nb); tsend[r] = R[r]; }
    else b_send(&c->b, r, r - 1, tsend[r], nb);
  }
  deliver(c, rets);
  for (int r = 0; r < P; r++) if (tsend[r] != R[r] && nb) memcpy(R[r], tsend[r], nb);
  free_ranks(inpl, P); free(tsend); free(newrank);
}

/* COLL_BASE_COMPUTE_BLOCKCOUNT, libbine_utils.h:63-69 */
static void blockcount(size_t count, int nblocks, int *split, size_t *early, size_t *late) {
  *early = *late = count / (size_t)nblocks;
  *split = (int)(count % (size_t)nblocks);
  if (*split) *early += 1;
}

/* allreduce_ring, :138-319 */
static void ar_ring(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  if (P == 1) { if (nb) memcpy(R[0], S[0], nb); return; }
  if (count < (size_t)P) { ar_recursivedoubling(c, count, S, R, rets); return; }
  int split; size_t early, late;
  blockcount(count, P, &split, &early, &late);
  size_t maxseg = early;
#define BOFF(b) ((b) < split ? (size_t)(b) * early : (size_t)(b) * late + (size_t)split)
#define BCNT(b) ((b) < split ? early : late)
  char **inbuf0 = alloc_ranks(P, maxseg * esz), **inbuf1 = alloc_ranks(P, maxseg * esz);
  char **inbuf[2] = {inbuf0, inbuf1};
  for (int r = 0; r < P; r++) memcpy(R[r], S[r], nb);
  int inbi = 0;
  for (int r = 0; r < P; r++) {                                      /* :226-235 */
    b_recv(&c->b, r, (r + P - 1) % P, inbuf[inbi][r], maxseg * esz);
    b_send(&c->b, r, (r + 1) % P, EL(R[r], BOFF(r)), BCNT(r) * esz);
  }
  deliver(c, rets);
  for (int k = 2; k < P; k++) {                                      /* :237-263 */
    inbi ^= 1;
    for (int r = 0; r < P; r++) {
      int prev = (r + P - k + 1) % P;
      red(c, inbuf[inbi ^ 1][r], EL(R[r], BOFF(prev)), BCNT(prev));
      b_recv(&c->b, r, (r + P - 1) % P, inbuf[inbi][r], maxseg * esz);
      b_send(&c->b, r, (r + 1) % P, EL(R[r], BOFF(prev)), BCNT(prev) * esz);
    }
    deliver(c, rets);
  }
  for (int r = 0; r < P; r++) {                                      /* :265-277 */
    int from = (r + 1) % P;
    red(c, inbuf[inbi][r], EL(R[r], BOFF(from)), BCNT(from));
  }
  for (int k = 0; k < P - 1; k++) {                                  /* :282-304 */
    for (int r = 0; r < P; r++) {
      int rf = (r + P - k) % P, sf = (r + 1 + P - k) % P;
      b_send(&c->b, r, (r + 1) % P, EL(R[r], BOFF(sf)), BCNT(sf) * esz);
      b_recv(&c->b, r, (r + P - 1) % P, EL(R[r], BOFF(rf)), maxseg * esz);
    }
    deliver(c, rets);
  }
#undef BOFF
#undef BCNT
  free_ranks(inbuf0, P); free_ranks(inbuf1, P);
}

/* allreduce_rabenseifner, :441-694 */
static void ar_rabenseifner(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  int steps = hibit(P, 31);
  int adj = 1 << steps, rem = P - adj;
  char **tmp = alloc_ranks(P, nb);
  int *vrank = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) if (nb) memcpy(R[r], S[r], nb);
  int lh = (int)(count / 2), rh = (int)count - lh;
  for (int r = 0; r < P; r++) {                                      /* :502-553 */
    if (r < 2 * rem) {
      if (r % 2) {
        b_send(&c->b, r, r - 1, R[r], (size_t)lh * esz);
        b_recv(&c->b, r, r - 1, EL(tmp[r], lh), (size_t)rh * esz);
      } else {
        b_send(&c->b, r, r + 1, EL(R[r], lh), (size_t)rh * esz);
        b_recv(&c->b, r, r + 1, tmp[r], (size_t)lh * esz);
      }
    }
  }
  deliver(c, rets);
  for (int r = 0; r < 2 * rem; r++) {
    if (r % 2) { red(c, EL(tmp[r], lh), EL(R[r], lh), (size_t)rh); b_send(&c->b, r, r - 1, EL(R[r], lh), (size_t)rh * esz); vrank[r] = -1; }
    else { red(c, tmp[r], R[r], (size_t)lh); b_recv(&c->b, r, r + 1, EL(R[r], lh), (size_t)rh * esz); vrank[r] = r / 2; }
  }
  deliver(c, rets);
  for (int r = 2 * rem; r < P; r++) vrank[r] = r - rem;
  int *rindex = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *sindex = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *rcount = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *scount = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *wsize = (int *)malloc(sizeof(int) * (size_t)P);
  int *stp = (int *)calloc((size_t)P, sizeof(int));
#define IX(a, r, s) a[(r) * (steps + 1) + (s)]
  for (int r = 0; r < P; r++) wsize[r] = (int)count;
  for (int mask = 1; mask < adj; mask <<= 1) {                       /* :581-630 */
    for (int r = 0; r < P; r++) {
      if (vrank[r] == -1) continue;
      int s = stp[r];
      int vdest = vrank[r] ^ mask;
      int dest = vdest < rem ? vdest * 2 : vdest + rem;
      if (r < dest) {
        IX(rcount, r, s) = wsize[r] / 2; IX(scount, r, s) = wsize[r] - IX(rcount, r, s);
        IX(sindex, r, s) = IX(rindex, r, s) + IX(rcount, r, s);
      } else {
        IX(scount, r, s) = wsize[r] / 2; IX(rcount, r, s) = wsize[r] - IX(scount, r, s);
        IX(rindex, r, s) = IX(sindex, r, s) + IX(scount, r, s);
      }
      b_send(&c->b, r, dest, EL(R[r], IX(sindex, r, s)), (size_t)IX(scount, r, s) * esz);
      b_recv(&c->b, r, dest, EL(tmp[r], IX(rindex, r, s)), (size_t)IX(rcount, r, s) * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      if (vrank[r] == -1) continue;
      int s = stp[r];
      red(c, EL(tmp[r], IX(rindex, r, s)), EL(R[r], IX(rindex, r, s)), (size_t)IX(rcount, r, s));
      if (s + 1 < steps) {
        IX(rindex, r, s + 1) = IX(rindex, r, s); IX(sindex, r, s + 1) = IX(rindex, r, s);
        wsize[r] = IX(rcount, r, s); stp[r] = s + 1;
      }
    }
  }
  for (int r = 0; r < P; r++) stp[r] = steps - 1;
  for (int mask = adj >> 1; mask > 0; mask >>= 1) {                  /* :644-661 */
    for (int r = 0; r < P; r++) {
      if (vrank[r] == -1) continue;
      int s = stp[r];
      int vdest = vrank[r] ^ mask;
      int dest = vdest < rem ? vdest * 2 : vdest + rem;
      b_send(&c->b, r, dest, EL(R[r], IX(rindex, r, s)), (size_t)IX(rcount, r, s) * esz);
      b_recv(&c->b, r, dest, EL(R[r], IX(sindex, r, s)), (size_t)IX(scount, r, s) * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) stp[r]--;
  }
#undef IX
  for (int r = 0; r < 2 * rem; r++) {                                /* :667-680 */
    if (r % 2) b_recv(&c->b, r, r - 1, R[r], nb);
    else b_send(&c->b, r, r + 1, R[r], nb);
  }
  deliver(c, rets);
  free_ranks(tmp, P); free(vrank); free(rindex); free(sindex); free(rcount); free(scount);
  free(wsize); free(stp);
}

/* allreduce_bine_lat, :321-439 */
static void ar_bine_lat(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  if (P == 1) { if (nb) memcpy(R[0], S[0], nb); return; }
  char **inpl = alloc_ranks(P, nb);
  char **tsend = (char **)malloc(sizeof(char *) * (size_t)P);
  int *nr = (int *)malloc(sizeof(int) * (size_t)P), *lf = (int *)calloc((size_t)P, sizeof(int));
  for (int r = 0; r < P; r++) { if (nb) memcpy(inpl[r], S[r], nb); tsend[r] = inpl[r]; }
  int steps = hibit(P, 31), adj = 1 << steps, extra = P - adj, pw2 = is_pow2(P);
  for (int r = 0; r < P; r++) {                                      /* :380-391 */
    nr[r] = r;
    if (r < 2 * extra) {
      if (r % 2 == 0) { b_send(&c->b, r, r + 1, tsend[r], nb); lf[r] = 1; }
      else { b_recv(&c->b, r, r - 1, R[r], nb); nr[r] = r >> 1; }
    } else nr[r] = r - extra;
  }
  deliver(c, rets);
  for (int r = 1; r < 2 * extra; r += 2) red(c, R[r], tsend[r], count);
  for (int s = 0; s < steps; s++) {                                  /* :396-411 */
    for (int r = 0; r < P; r++) {
      if (lf[r]) continue;
      int vd = orc_pi(nr[r], s, adj);
      int dest = pw2 ? vd : (vd < extra ? (vd << 1) + 1 : vd + extra);
      b_send(&c->b, r, dest, tsend[r], nb);
      b_recv(&c->b, r, dest, R[r], nb);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) if (!lf[r]) red(c, R[r], tsend[r], count);
  }
  for (int r = 0; r < 2 * extra; r++) {                              /* :415-424 */
    if (!lf[r]) b_send(&c->b, r, r - 1, tsend[r], nb);
    else { b_recv(&c->b, r, r + 1, R[r], nb); tsend[r] = R[r]; }
  }
  deliver(c, rets);
  for (int r = 0; r < P; r++) if (tsend[r] != R[r] && nb) memcpy(R[r], tsend[r], nb);
  free_ranks(inpl, P); free(tsend); free(nr); free(lf);
}

/* allreduce_bine_bdw_static, :696-817 (tables regenerated, see above) */
static void ar_bine_bdw_static(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  int split; size_t big, small;
  blockcount(count, P, &split, &big, &small);
  int *perm = (int *)malloc(sizeof(int) * (size_t)P);
  int *st = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps);
  int *rt = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps);
  orc_static_tables(P, perm, st, rt);
  char **tmp = alloc_ranks(P, nb);
  for (int r = 0; r < P; r++) if (nb) memcpy(R[r], S[r], nb);
#define WCNT(start, w) (((start) + (w) <= split) ? (size_t)(w) * big : ((start) >= split) ? (size_t)(w) * small : (size_t)(w) * small + (size_t)(split - (start)))
#define WOFF(start) (((start) <= split) ? (size_t)(start) * big : (size_t)(start) * small + (size_t)split)
  int w = P;
  for (int s = 0; s < steps; s++) {                                  /* :745-776 */
    w >>= 1;
    for (int r = 0; r < P; r++) {
      int dest = orc_pi(r, s, P), sb = st[r * steps + s], rb = rt[r * steps + s];
      b_send(&c->b, r, dest, EL(R[r], WOFF(sb)), WCNT(sb, w) * esz);
      b_recv(&c->b, r, dest, tmp[r], WCNT(rb, w) * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      int rb = rt[r * steps + s];
      red(c, tmp[r], EL(R[r], WOFF(rb)), WCNT(rb, w));
    }
  }
  for (int s = steps - 1; s >= 0; s--) {                             /* :779-809 */
    for (int r = 0; r < P; r++) {
      int dest = orc_pi(r, s, P), sb = st[r * steps + s], rb = rt[r * steps + s];
      b_send(&c->b, r, dest, EL(R[r], WOFF(rb)), WCNT(rb, w) * esz);
      b_recv(&c->b, r, dest, EL(R[r], WOFF(sb)), WCNT(sb, w) * esz);
    }
    deliver(c, rets);
    w <<= 1;
  }
#undef WCNT
#undef WOFF
  free_ranks(tmp, P); free(perm); free(st); free(rt);
}

/* allreduce_bine_bdw_remap, :820-923, and the power-of-two-adjusted,
 * optionally segmented variant allreduce_bine_bdw_remap_segmented,
 * :1093-1308.  seg = 0 -> plain remap semantics. */
static void ar_bine_remap_core(ctx_t *c, size_t count, char **S, char **R, int *rets,
                               int segmented, size_t segsize, int ref_bugs) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  int steps, adj, extra, pw2;
  if (!segmented) {
    steps = log_2(P);
    if (!is_pow2(P) || steps == -1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
    adj = P; extra = 0; pw2 = 1;
  } else {
    steps = hibit(P, 31);
    if (steps == -1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
    adj = 1 << steps; extra = P - adj; pw2 = is_pow2(P);
  }
  size_t segcount = segsize / esz;
  if (!segmented || segsize == 0) segcount = count;
  if (segmented && ref_bugs && segcount == 0) {     /* the reference divides by 0 here (:1211) */
    for (int r = 0; r < P; r++) rets[r] = ORC_ASSERT;
    return;
  }
  char **tmp = alloc_ranks(P, nb);
  int *nr = (int *)malloc(sizeof(int) * (size_t)P), *lf = (int *)calloc((size_t)P, sizeof(int));
  /* :1148-1169 fold for non-power-of-two sizes */
  for (int r = 0; r < P; r++) {
    nr[r] = r;
    if (r < 2 * extra) {
      if (r % 2 == 0) { b_send(&c->b, r, r + 1, S[r], nb); lf[r] = 1; }
      else { b_recv(&c->b, r, r - 1, R[r], nb); nr[r] = r >> 1; }
    } else {
      nr[r] = r - extra;
      if (nb) memcpy(R[r], S[r], nb);
    }
  }
  deliver(c, rets);
  for (int r = 1; r < 2 * extra; r += 2) red(c, S[r], R[r], count);  /* :1158 in=sbuf, inout=rbuf */
  int *ri = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *si = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *rc = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  int *sc = (int *)calloc((size_t)P * (size_t)(steps + 1), sizeof(int));
  size_t *w = (size_t *)malloc(sizeof(size_t) * (size_t)P);
  uint32_t *vr = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)P);
  int *dst = (int *)malloc(sizeof(int) * (size_t)P);
#define IX(a, r, s) a[(r) * (steps + 1) + (s)]
  for (int r = 0; r < P; r++) { w[r] = count; vr[r] = orc_remap_rank((uint32_t)adj, (uint32_t)nr[r]); }
  for (int s = 0; s < steps; s++) {
    size_t maxph = 0;
    int *nph = (int *)calloc((size_t)P, sizeof(int));
    for (int r = 0; r < P; r++) {                                    /* :868-880 / :1188-1209 */
      if (lf[r]) continue;
      int vd = orc_pi(nr[r], s, adj);
      dst[r] = pw2 ? vd : (vd < extra ? (vd << 1) + 1 : vd + extra);
      uint32_t vdest = orc_remap_rank((uint32_t)adj, (uint32_t)vd);
      if (vr[r] < vdest) {
        IX(rc, r, s) = (int)(w[r] / 2); IX(sc, r, s) = (int)(w[r] - (size_t)IX(rc, r, s));
        IX(si, r, s) = IX(ri, r, s) + IX(rc, r, s);
      } else {
        IX(sc, r, s) = (int)(w[r] / 2); IX(rc, r, s) = (int)(w[r] - (size_t)IX(sc, r, s));
        IX(ri, r, s) = IX(si, r, s) + IX(sc, r, s);
      }
    }
    if (!segmented || !ref_bugs) {
      /* one exchange of the whole window, one reduce (:882-888); the segmented
       * variant computes the same values when its tail is handled */
      for (int r = 0; r < P; r++) {
        if (lf[r]) continue;
        b_send(&c->b, r, dst[r], EL(R[r], IX(si, r, s)), (size_t)IX(sc, r, s) * esz);
        b_recv(&c->b, r, dst[r], tmp[r], (size_t)IX(rc, r, s) * esz);
      }
      deliver(c, rets);
      for (int r = 0; r < P; r++)
        if (!lf[r]) red(c, tmp[r], EL(R[r], IX(ri, r, s)), (size_t)IX(rc, r, s));
    } else {
      /* :1211-1253 verbatim phase structure, including the unreduced tail */
      for (int r = 0; r < P; r++) {
        if (lf[r]) continue;
        int rcn = IX(rc, r, s), scn = IX(sc, r, s);
        nph[r] = rcn > scn ? (int)((size_t)rcn / segcount) : (int)((size_t)scn / segcount);
        if ((size_t)(nph[r] > 1 ? nph[r] : 1) > maxph) maxph = (size_t)(nph[r] > 1 ? nph[r] : 1);
      }
      for (size_t ph = 0; ph < maxph; ph++) {
        for (int r = 0; r < P; r++) {
          if (lf[r]) continue;
          int np = nph[r] > 1 ? nph[r] : 1;
          if ((int)ph >= np) continue;
          size_t pscn = (size_t)IX(sc, r, s) > segcount ? segcount : (size_t)IX(sc, r, s);
          size_t prcn = (size_t)IX(rc, r, s) > segcount ? segcount : (size_t)IX(rc, r, s);
          b_send(&c->b, r, dst[r], EL(R[r], (size_t)IX(si, r, s) + ph * pscn), pscn * esz);
          b_recv(&c->b, r, dst[r], tmp[r], prcn * esz);
        }
        deliver(c, rets);
        for (int r = 0; r < P; r++) {
          if (lf[r]) continue;
          int np = nph[r] > 1 ? nph[r] : 1;
          if ((int)ph >= np) continue;
          size_t prcn = (size_t)IX(rc, r, s) > segcount ? segcount : (size_t)IX(rc, r, s);
          red(c, tmp[r], EL(R[r], (size_t)IX(ri, r, s) + ph * prcn), prcn);
        }
      }
    }
    free(nph);
    for (int r = 0; r < P; r++) {                                    /* :890-894 */
      if (lf[r]) continue;
      if (s + 1 < steps) { IX(ri, r, s + 1) = IX(ri, r, s); IX(si, r, s + 1) = IX(ri, r, s); w[r] = (size_t)IX(rc, r, s); }
    }
  }
  for (int s = steps - 1; s >= 0; s--) {                             /* :898-907 / :1263-1277 */
    for (int r = 0; r < P; r++) {
      if (lf[r]) continue;
      int vd = orc_pi(nr[r], s, adj);
      int d = pw2 ? vd : (vd < extra ? (vd << 1) + 1 : vd + extra);
      b_send(&c->b, r, d, EL(R[r], IX(ri, r, s)), (size_t)IX(rc, r, s) * esz);
      b_recv(&c->b, r, d, EL(R[r], IX(si, r, s)), (size_t)IX(sc, r, s) * esz);
    }
    deliver(c, rets);
  }
#undef IX
  for (int r = 0; r < 2 * extra; r++) {                              /* :1282-1290 */
    if (!lf[r]) b_send(&c->b, r, r - 1, R[r], nb);
    else b_recv(&c->b, r, r + 1, R[r], nb);
  }
  deliver(c, rets);
  free_ranks(tmp, P); free(nr); free(lf); free(ri); free(si); free(rc); free(sc); free(w); free(vr); free(dst);
}

/* allreduce_bine_block_by_block_any_even, :925-1091 */
static void ar_bine_bbb_any_even(ctx_t *c, size_t count, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (P % 2) { for (int r = 0; r < P; r++) rets[r] = ORC_ASSERT; return; }  /* :931 */
  int *displs = (int *)malloc(sizeof(int) * (size_t)P), *rcnt = (int *)malloc(sizeof(int) * (size_t)P);
  int cpb = (int)(count / (size_t)P), sofar = 0;
  for (int i = 0; i < P; i++) {
    displs[i] = sofar;
    rcnt[i] = (size_t)i < count % (size_t)P ? cpb + 1 : cpb;
    sofar += rcnt[i];
  }
  char **tmp = alloc_ranks(P, count * esz);
  for (int r = 0; r < P; r++) memcpy(R[r], S[r], count * esz);
  int **btr = (int **)malloc(sizeof(int *) * (size_t)P);
  int *nrr = (int *)calloc((size_t)P, sizeof(int));
  for (int r = 0; r < P; r++) btr[r] = (int *)malloc(sizeof(int) * (size_t)P);
  int mask = 1, rstep = log_2(P) - 1;
  while (mask < P) {                                                 /* :957-1019 */
    for (int r = 0; r < P; r++) {
      int partner = r % 2 == 0 ? mod(r + nb2b((uint32_t)((mask << 1) - 1)), P)
                               : mod(r - nb2b((uint32_t)((mask << 1) - 1)), P);
      nrr[r] = 0;
      for (int block = 1; block < P; block++) {
        int k = 31 - __builtin_clz(orc_get_nu((uint32_t)block, (uint32_t)P));
        if (k != rstep) continue;
        int bts, brv;
        if (r % 2 == 0) { bts = mod(block + r, P); brv = mod(partner - block, P); }
        else { bts = mod(r - block, P); brv = mod(block + partner, P); }
        if (bts != r) b_send(&c->b, r, partner, EL(R[r], displs[bts]), (size_t)rcnt[bts] * esz);
        if (brv != partner) {
          btr[r][nrr[r]++] = brv;
          b_recv(&c->b, r, partner, EL(tmp[r], displs[brv]), (size_t)rcnt[brv] * esz);
        }
      }
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++)
      for (int i = 0; i < nrr[r]; i++) {
        int b = btr[r][i];
        red(c, EL(tmp[r], displs[b]), EL(R[r], displs[b]), (size_t)rcnt[b]);
      }
    mask <<= 1; rstep--;
  }
  int step = 0;
  mask >>= 1;
  while (mask > 0) {                                                 /* :1024-1072 */
    for (int r = 0; r < P; r++) {
      int partner = r % 2 == 0 ? mod(r + nb2b((uint32_t)((mask << 1) - 1)), P)
                               : mod(r - nb2b((uint32_t)((mask << 1) - 1)), P);
      for (int block = 1; block < P; block++) {
        int k = 31 - __builtin_clz(orc_get_nu((uint32_t)block, (uint32_t)P));
        if (!(k == step || block == 0)) continue;
        int bts, brv;
        if (r % 2 == 0) { brv = mod(block + r, P); bts = mod(partner - block, P); }
        else { brv = mod(r - block, P); bts = mod(block + partner, P); }
        b_send(&c->b, r, bts != partner ? partner : -1, EL(R[r], displs[bts]), (size_t)rcnt[bts] * esz);
        b_recv(&c->b, r, brv != r ? partner : -1, EL(R[r], displs[brv]), (size_t)rcnt[brv] * esz);
      }
    }
    deliver(c, rets);
    mask >>= 1; step++;
  }
  for (int r = 0; r < P; r++) free(btr[r]);
  free(btr); free(nrr); free(displs); free(rcnt); free_ranks(tmp, P);
}

int orc_allreduce(const char *algo, int P, size_t count, int dtype, int op,
                  size_t segsize, int ref_bugs,
                  const void *const *sbufs, void *const *rbufs, int *rets) {
  if (P < 1 || !orc_dtype_size(dtype)) return -1;
  ctx_t c; memset(&c, 0, sizeof c);
  c.P = P; c.dtype = dtype; c.op = op; c.esz = orc_dtype_size(dtype);
  char **S = (char **)sbufs, **R = (char **)rbufs;
  for (int r = 0; r < P; r++) rets[r] = ORC_OK;
  int known = 1;
  if (!strcmp(algo, "recursivedoubling")) ar_recursivedoubling(&c, count, S, R, rets);
  else if (!strcmp(algo, "ring")) ar_ring(&c, count, S, R, rets);
  else if (!strcmp(algo, "rabenseifner")) ar_rabenseifner(&c, count, S, R, rets);
  else if (!strcmp(algo, "bine_lat")) ar_bine_lat(&c, count, S, R, rets);
  else if (!strcmp(algo, "bine_bdw_static")) ar_bine_bdw_static(&c, count, S, R, rets);
  else if (!strcmp(algo, "bine_bdw_remap")) ar_bine_remap_core(&c, count, S, R, rets, 0, 0, 0);
  else if (!strcmp(algo, "bine_bdw_remap_segmented")) ar_bine_remap_core(&c, count, S, R, rets, 1, segsize, ref_bugs);
  else if (!strcmp(algo, "bine_block_by_block_any_even")) ar_bine_bbb_any_even(&c, count, S, R, rets);
  else known = 0;
  if (c.dead) for (int r = 0; r < P; r++) if (rets[r] == ORC_OK) rets[r] = c.dead;
  b_free(&c.b);
  return known ? 0 : -1;
}

/* ----------------------------------------------------------------------- */
/* reduce_scatter -- libbine_reduce_scatter.c                                */
/* ----------------------------------------------------------------------- */

/* reduce_scatter_recursivehalving, :15-257 */
static void rs_recursivehalving(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  ptrdiff_t *disps = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)P);
  disps[0] = 0;
  for (int i = 0; i < P - 1; i++) disps[i + 1] = disps[i] + rc[i];
  size_t count = (size_t)(disps[P - 1] + rc[P - 1]);
  if (!count) { free(disps); return; }
  char **rb = alloc_ranks(P, count * esz), **res = alloc_ranks(P, count * esz);
  for (int r = 0; r < P; r++) memcpy(res[r], S[r], count * esz);
  int tsz = next_pow2(P) >> 1, rem = P - tsz;
  int *tr = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) {                                      /* :84-104 */
    if (r < 2 * rem) {
      if ((r & 1) == 0) { b_send(&c->b, r, r + 1, res[r], count * esz); tr[r] = -1; }
      else { b_recv(&c->b, r, r - 1, rb[r], count * esz); tr[r] = r / 2; }
    } else tr[r] = r - rem;
  }
  deliver(c, rets);
  for (int r = 1; r < 2 * rem; r += 2) red(c, rb[r], res[r], count);
  size_t *trc = (size_t *)malloc(sizeof(size_t) * (size_t)tsz);
  ptrdiff_t *tds = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)tsz);
  for (int i = 0; i < tsz; i++) trc[i] = i < rem ? (size_t)(rc[i * 2 + 1] + rc[i * 2]) : (size_t)rc[i + rem];
  tds[0] = 0;
  for (int i = 0; i < tsz - 1; i++) tds[i + 1] = tds[i] + (ptrdiff_t)trc[i];
  int *sidx = (int *)calloc((size_t)P, sizeof(int)), *ridx = (int *)calloc((size_t)P, sizeof(int));
  int *last = (int *)malloc(sizeof(int) * (size_t)P);
  size_t *rcn = (size_t *)calloc((size_t)P, sizeof(size_t));
  for (int r = 0; r < P; r++) last[r] = tsz;
  for (int mask = tsz >> 1; mask > 0; mask >>= 1) {                  /* :149-217 */
    for (int r = 0; r < P; r++) {
      if (tr[r] < 0) continue;
      int tp = tr[r] ^ mask;
      int peer = tp < rem ? tp * 2 + 1 : tp + rem;
      size_t scn = 0; rcn[r] = 0;
      if (tr[r] < tp) {
        sidx[r] = ridx[r] + mask;
        for (int i = sidx[r]; i < last[r]; i++) scn += trc[i];
        for (int i = ridx[r]; i < sidx[r]; i++) rcn[r] += trc[i];
      } else {
        ridx[r] = sidx[r] + mask;
        for (int i = sidx[r]; i < ridx[r]; i++) scn += trc[i];
        for (int i = ridx[r]; i < last[r]; i++) rcn[r] += trc[i];
      }
      if (rcn[r] > 0) b_recv(&c->b, r, peer, EL(rb[r], tds[ridx[r]]), rcn[r] * esz);
      if (scn > 0) b_send(&c->b, r, peer, EL(res[r], tds[sidx[r]]), scn * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      if (tr[r] < 0) continue;
      if (rcn[r] > 0) red(c, EL(rb[r], tds[ridx[r]]), EL(res[r], tds[ridx[r]]), rcn[r]);
      sidx[r] = ridx[r];
      last[r] = ridx[r] + mask;
    }
  }
  for (int r = 0; r < P; r++)                                        /* :220-228 */
    if (tr[r] >= 0 && rc[r]) memcpy(R[r], EL(res[r], disps[r]), (size_t)rc[r] * esz);
  for (int r = 0; r < 2 * rem; r++) {                                /* :236-249 */
    if ((r & 1) == 0) { if (rc[r]) b_recv(&c->b, r, r + 1, R[r], (size_t)rc[r] * esz); }
    else if (rc[r - 1]) b_send(&c->b, r, r - 1, EL(res[r], disps[r - 1]), (size_t)rc[r - 1] * esz);
  }
  deliver(c, rets);
  free(disps); free_ranks(rb, P); free_ranks(res, P); free(tr); free(trc); free(tds);
  free(sidx); free(ridx); free(last); free(rcn);
}

/* reduce_scatter_recursive_distance_doubling, :259-419 */
static void rs_recursive_distance_doubling(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps == -1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  ptrdiff_t *disps = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)P);
  disps[0] = 0;
  for (int i = 0; i < P - 1; i++) disps[i + 1] = disps[i] + rc[i];
  size_t count = (size_t)(disps[P - 1] + rc[P - 1]);
  if (!count) { free(disps); return; }
  char **rb = alloc_ranks(P, count * esz), **res = alloc_ranks(P, count * esz);
  for (int r = 0; r < P; r++) memcpy(res[r], S[r], count * esz);
  int *sidx = (int *)calloc((size_t)P, sizeof(int)), *ridx = (int *)calloc((size_t)P, sizeof(int));
  int *last = (int *)malloc(sizeof(int) * (size_t)P);
  size_t *rcn = (size_t *)calloc((size_t)P, sizeof(size_t));
  for (int r = 0; r < P; r++) last[r] = P;
  int w = P >> 1, dist = 1;
  for (int s = 0; s < steps; s++) {                                  /* :328-385 */
    for (int r = 0; r < P; r++) {
      int peer = r ^ dist;
      size_t scn = 0; rcn[r] = 0;
      if (r < peer) {
        sidx[r] = ridx[r] + w;
        for (int i = sidx[r]; i < last[r]; i++) scn += (size_t)rc[i];
        for (int i = ridx[r]; i < sidx[r]; i++) rcn[r] += (size_t)rc[i];
      } else {
        ridx[r] = sidx[r] + w;
        for (int i = sidx[r]; i < ridx[r]; i++) scn += (size_t)rc[i];
        for (int i = ridx[r]; i < last[r]; i++) rcn[r] += (size_t)rc[i];
      }
      if (rcn[r] > 0) b_recv(&c->b, r, peer, EL(rb[r], disps[ridx[r]]), rcn[r] * esz);
      if (scn > 0) b_send(&c->b, r, peer, EL(res[r], disps[sidx[r]]), scn * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      if (rcn[r] > 0) red(c, EL(rb[r], disps[ridx[r]]), EL(res[r], disps[ridx[r]]), rcn[r]);
      sidx[r] = ridx[r];
      last[r] = ridx[r] + w;
    }
    w >>= 1; dist <<= 1;
  }
  for (int r = 0; r < P; r++) {                                      /* :394-410 */
    int inv = (int)inverse_rank((uint32_t)P, (uint32_t)r);
    if (r != inv) {
      b_send(&c->b, r, inv, EL(res[r], disps[inv]), (size_t)rc[inv] * esz);
      b_recv(&c->b, r, inv, R[r], (size_t)rc[r] * esz);
    } else if (rc[r]) memcpy(R[r], EL(res[r], disps[r]), (size_t)rc[r] * esz);
  }
  deliver(c, rets);
  free(disps); free_ranks(rb, P); free_ranks(res, P); free(sidx); free(ridx); free(last); free(rcn);
}

/* reduce_scatter_ring, :421-572 */
static void rs_ring(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  ptrdiff_t *displs = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)P);
  size_t total = (size_t)rc[0], maxb = (size_t)rc[0];
  displs[0] = 0;
  for (int i = 1; i < P; i++) { displs[i] = (ptrdiff_t)total; total += (size_t)rc[i]; if (maxb < (size_t)rc[i]) maxb = (size_t)rc[i]; }
  if (P == 1) { if (total) memcpy(R[0], S[0], total * esz); free(displs); return; }
  char **acc = alloc_ranks(P, total * esz);
  char **ib[2] = {alloc_ranks(P, maxb * esz), alloc_ranks(P, maxb * esz)};
  for (int r = 0; r < P; r++) memcpy(acc[r], S[r], total * esz);
  int inbi = 0;
  for (int r = 0; r < P; r++) {                                      /* :509-518 */
    int from = (r + P - 1) % P;
    b_recv(&c->b, r, from, ib[inbi][r], maxb * esz);
    b_send(&c->b, r, (r + 1) % P, EL(acc[r], displs[from]), (size_t)rc[from] * esz);
  }
  deliver(c, rets);
  for (int k = 2; k < P; k++) {                                      /* :520-542 */
    inbi ^= 1;
    for (int r = 0; r < P; r++) {
      int prev = (r + P - k) % P;
      b_recv(&c->b, r, (r + P - 1) % P, ib[inbi][r], maxb * esz);
      red(c, ib[inbi ^ 1][r], EL(acc[r], displs[prev]), (size_t)rc[prev]);
      b_send(&c->b, r, (r + 1) % P, EL(acc[r], displs[prev]), (size_t)rc[prev] * esz);
    }
    deliver(c, rets);
  }
  for (int r = 0; r < P; r++) {                                      /* :545-555 */
    red(c, ib[inbi][r], EL(acc[r], displs[r]), (size_t)rc[r]);
    if (rc[r]) memcpy(R[r], EL(acc[r], displs[r]), (size_t)rc[r] * esz);
  }
  free(displs); free_ranks(acc, P); free_ranks(ib[0], P); free_ranks(ib[1], P);
}

/* sum_counts, libbine_utils.h:404-410 */
static size_t sum_counts(const int *counts, const ptrdiff_t *displs, int rem, int lo, int hi) {
  lo = lo < rem ? lo * 2 : lo + rem;
  hi = hi < rem ? hi * 2 + 1 : hi + rem;
  return (size_t)(displs[hi] + counts[hi] - displs[lo]);
}

/* reduce_scatter_butterfly, :575-761 */
static void rs_butterfly(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (P < 2) return;                                                 /* :585-586: rbuf untouched */
  ptrdiff_t *displs = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)P);
  displs[0] = 0;
  for (int i = 1; i < P; i++) displs[i] = displs[i - 1] + rc[i - 1];
  size_t total = (size_t)(displs[P - 1] + rc[P - 1]);
  char **ba = alloc_ranks(P, total * esz), **bb = alloc_ranks(P, total * esz);
  char **ps = (char **)malloc(sizeof(char *) * (size_t)P), **pr = (char **)malloc(sizeof(char *) * (size_t)P);
  for (int r = 0; r < P; r++) { ps[r] = ba[r]; pr[r] = bb[r]; memcpy(ps[r], S[r], total * esz); }
  int pof2 = next_pow2(P) >> 1, rem = P - pof2, l2 = log_2(pof2);
  int *vr = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) {                                      /* :638-656 */
    if (r < 2 * rem) {
      if (r % 2 == 0) { b_send(&c->b, r, r + 1, ps[r], total * esz); vr[r] = -1; }
      else { b_recv(&c->b, r, r - 1, pr[r], total * esz); vr[r] = r / 2; }
    } else vr[r] = r - rem;
  }
  deliver(c, rets);
  for (int r = 1; r < 2 * rem; r += 2) red(c, pr[r], ps[r], total);
  int *si = (int *)calloc((size_t)P, sizeof(int)), *ri = (int *)calloc((size_t)P, sizeof(int));
  ptrdiff_t *rd = (ptrdiff_t *)calloc((size_t)P, sizeof(ptrdiff_t));
  size_t *rcn = (size_t *)calloc((size_t)P, sizeof(size_t));
  int nblocks = pof2;
  for (int mask = 1; mask < pof2; mask <<= 1) {                      /* :671-714 */
    nblocks /= 2;
    for (int r = 0; r < P; r++) {
      if (vr[r] == -1) continue;
      int vp = vr[r] ^ mask, peer = vp < rem ? vp * 2 + 1 : vp + rem;
      if ((vr[r] & mask) == 0) si[r] += nblocks; else ri[r] += nblocks;
      size_t scn = sum_counts(rc, displs, rem, si[r], si[r] + nblocks - 1);
      int ix = si[r] < rem ? 2 * si[r] : rem + si[r];
      ptrdiff_t sd = displs[ix];
      rcn[r] = sum_counts(rc, displs, rem, ri[r], ri[r] + nblocks - 1);
      ix = ri[r] < rem ? 2 * ri[r] : rem + ri[r];
      rd[r] = displs[ix];
      b_send(&c->b, r, peer, EL(ps[r], sd), scn * esz);
      b_recv(&c->b, r, peer, EL(pr[r], rd[r]), rcn[r] * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      if (vr[r] == -1) continue;
      int vp = vr[r] ^ mask;
      if (vr[r] < vp) {
        red(c, EL(ps[r], rd[r]), EL(pr[r], rd[r]), rcn[r]);
        char *t = ps[r]; ps[r] = pr[r]; pr[r] = t;
      } else red(c, EL(pr[r], rd[r]), EL(ps[r], rd[r]), rcn[r]);
      si[r] = ri[r];
    }
  }
  for (int r = 0; r < P; r++) {                                      /* :719-751 */
    if (vr[r] != -1) {
      int vp = (int)mirror_perm((uint32_t)vr[r], l2);
      int peer = vp < rem ? vp * 2 + 1 : vp + rem;
      int ix = si[r] < rem ? 2 * si[r] : rem + si[r];
      if (vp < rem) b_send(&c->b, r, peer - 1, EL(ps[r], displs[ix]), (size_t)rc[ix] * esz);
      if (vp < rem) ix++;
      if (vp != vr[r]) {
        b_send(&c->b, r, peer, EL(ps[r], displs[ix]), (size_t)rc[ix] * esz);
        b_recv(&c->b, r, peer, R[r], (size_t)rc[r] * esz);
      } else if (rc[r]) memcpy(R[r], EL(ps[r], displs[r]), (size_t)rc[r] * esz);
    } else {
      int vp = (int)mirror_perm((uint32_t)((r + 1) / 2), l2);
      int peer = vp < rem ? vp * 2 + 1 : vp + rem;
      b_recv(&c->b, r, peer, R[r], (size_t)rc[r] * esz);
    }
  }
  deliver(c, rets);
  free(displs); free_ranks(ba, P); free_ranks(bb, P); free(ps); free(pr); free(vr);
  free(si); free(ri); free(rd); free(rcn);
}

/* reduce_scatter_bine_static, :763-904 */
static void rs_bine_static(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  ptrdiff_t *disps = (ptrdiff_t *)malloc(sizeof(ptrdiff_t) * (size_t)P);
  disps[0] = 0;
  for (int i = 0; i < P - 1; i++) disps[i + 1] = disps[i] + rc[i];
  size_t count = (size_t)(disps[P - 1] + rc[P - 1]);
  if (!count) { free(disps); return; }
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_SIZE; free(disps); return; }
  int *perm = (int *)malloc(sizeof(int) * (size_t)P);
  int *st = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps);
  int *rt = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps);
  orc_static_tables(P, perm, st, rt);
  char **rb = alloc_ranks(P, count * esz), **res = alloc_ranks(P, count * esz);
  for (int r = 0; r < P; r++) memcpy(res[r], S[r], count * esz);
  int w = P >> 1;
  size_t *rcn = (size_t *)calloc((size_t)P, sizeof(size_t));
  for (int s = 0; s < steps; s++) {                                  /* :839-877 */
    for (int r = 0; r < P; r++) {
      int peer = orc_pi(r, s, P), sb = st[r * steps + s], rbi = rt[r * steps + s];
      size_t scn = 0; rcn[r] = 0;
      for (int i = 0; i < w; i++) { scn += (size_t)rc[sb + i]; rcn[r] += (size_t)rc[rbi + i]; }
      b_send(&c->b, r, peer, EL(res[r], disps[sb]), scn * esz);
      b_recv(&c->b, r, peer, EL(rb[r], disps[rbi]), rcn[r] * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      int rbi = rt[r * steps + s];
      if (rcn[r] > 0) red(c, EL(rb[r], disps[rbi]), EL(res[r], disps[rbi]), rcn[r]);
    }
    w >>= 1;
  }
  for (int r = 0; r < P; r++) {                                      /* :880-896 */
    if (r != perm[r]) {
      int sender = -1;
      for (int j = 0; j < P; j++) if (perm[j] == r) { sender = j; break; }
      b_send(&c->b, r, perm[r], EL(res[r], disps[rt[r * steps + steps - 1]]), (size_t)rc[perm[r]] * esz);
      b_recv(&c->b, r, sender, R[r], (size_t)rc[r] * esz);
    } else if (rc[r]) memcpy(R[r], EL(res[r], disps[r]), (size_t)rc[r] * esz);
  }
  deliver(c, rets);
  free(disps); free(perm); free(st); free(rt); free_ranks(rb, P); free_ranks(res, P); free(rcn);
}

/* partner of the negabinary-distance Bine steps used by the send/permute
 * remap and block-by-block variants (e.g. libbine_reduce_scatter.c:936-940) */
static int nb_partner(int r, int mask, int P) {
  int d = nb2b((uint32_t)((mask << 1) - 1));
  return r % 2 == 0 ? mod(r + d, P) : mod(r - d, P);
}

/* reduce_scatter_bine_send_remap (:906-983) and _permute_remap (:985-1063) */
static void rs_bine_remap(ctx_t *c, const int *rc, char **S, char **R, int *rets, int permute) {
  int P = c->P; size_t esz = c->esz;
  if (!is_pow2(P)) {
    /* the reference has no power-of-two check here and hangs or crashes at
     * P = 3, 5, 6, 7 (no vector); reported as MPI_ERR_ARG,
     * the status the device path returns (deviations) */
    for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG;
    return;
  }
  if (permute)
    for (int i = 1; i < P; i++)
      if (rc[i] != rc[0]) {
        /* unequal blocks: the reference copies block i into block remap(i)'s
         * slot with block i's size (:1008-1011) and overruns its buffers --
         * undefined behaviour, no vector exists.  Reported as MPI_ERR_ARG, the
         * status the device path returns (deviations). */
        for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG;
        return;
      }
  int *displs = (int *)malloc(sizeof(int) * (size_t)P), count = 0;
  for (int i = 0; i < P; i++) { displs[i] = count; count += rc[i]; }
  char **tmp = alloc_ranks(P, (size_t)count * esz), **res = alloc_ranks(P, (size_t)count * esz);
  for (int r = 0; r < P; r++) {
    if (!permute) memcpy(res[r], S[r], (size_t)count * esz);
    else
      for (int i = 0; i < P; i++) {                                  /* :1008-1011 */
        int rr = (int)orc_remap_rank((uint32_t)P, (uint32_t)i);
        memcpy(EL(res[r], displs[rr]), EL(S[r], displs[i]), (size_t)rc[i] * esz);
      }
  }
  int mask = 1;
  int inv = (int)(1u << ((unsigned)(log_2(P) - 1) & 31u));
  int bfm = (int)~((unsigned)inv - 1u);
  while (mask < P) {                                                 /* :934-962 / :1017-1046 */
    for (int r = 0; r < P; r++) {
      int partner = nb_partner(r, mask, P);
      int sbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
      int scn = displs[sbl] - displs[sbf] + rc[sbl];
      int rbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)r) & bfm, rbl = rbf + inv - 1;
      int rcn = displs[rbl] - displs[rbf] + rc[rbl];
      b_send(&c->b, r, partner, EL(res[r], displs[sbf]), (size_t)scn * esz);
      b_recv(&c->b, r, partner, EL(tmp[r], displs[rbf]), (size_t)rcn * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      int rbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)r) & bfm, rbl = rbf + inv - 1;
      int rcn = displs[rbl] - displs[rbf] + rc[rbl];
      red(c, EL(tmp[r], displs[rbf]), EL(res[r], displs[rbf]), (size_t)rcn);
    }
    mask <<= 1; inv >>= 1; bfm >>= 1;
  }
  for (int r = 0; r < P; r++) {
    int rr = (int)orc_remap_rank((uint32_t)P, (uint32_t)r);
    if (!permute) {                                                  /* :966-969 */
      b_send(&c->b, r, rr, EL(res[r], displs[rr]), (size_t)rc[rr] * esz);
      b_recv(&c->b, r, ANY_SRC, R[r], (size_t)rc[r] * esz);
    } else if (rc[r]) memcpy(R[r], EL(res[r], displs[rr]), (size_t)rc[r] * esz);  /* :1049 */
  }
  deliver(c, rets);
  free(displs); free_ranks(tmp, P); free_ranks(res, P);
}

/* reduce_scatter_bine_block_by_block, :1066-1174 */
static void rs_bine_bbb(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (!is_pow2(P)) {
    /* no power-of-two check in the reference: it hangs at P = 3 (measured)
     * and indexes past its blocks; MPI_ERR_ARG, as the device path */
    for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG;
    return;
  }
  int *displs = (int *)malloc(sizeof(int) * (size_t)P), *invr = (int *)malloc(sizeof(int) * (size_t)P), count = 0;
  for (int i = 0; i < P; i++) { displs[i] = count; count += rc[i]; invr[orc_remap_rank((uint32_t)P, (uint32_t)i)] = i; }
  char **tmp = alloc_ranks(P, (size_t)count * esz), **res = alloc_ranks(P, (size_t)count * esz);
  for (int r = 0; r < P; r++) memcpy(res[r], S[r], (size_t)count * esz);
  int mask = 1;
  int inv = (int)(1u << ((unsigned)(log_2(P) - 1) & 31u));
  int bfm = (int)~((unsigned)inv - 1u);
  while (mask < P) {                                                 /* :1098-1156 */
    int lastst = (mask << 1) >= P;
    for (int r = 0; r < P; r++) {
      int partner = nb_partner(r, mask, P);
      int sbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
      int rbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)r) & bfm, rbl = rbf + inv - 1;
      for (int b = rbf; b <= rbl; b++)
        b_recv(&c->b, r, partner, lastst ? R[r] : EL(tmp[r], displs[invr[b]]), (size_t)rc[invr[b]] * esz);
      for (int b = sbf; b <= sbl; b++)
        b_send(&c->b, r, partner, EL(res[r], displs[invr[b]]), (size_t)rc[invr[b]] * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) {
      int rbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)r) & bfm, rbl = rbf + inv - 1;
      for (int b = rbf; b <= rbl; b++) {
        if (lastst) red(c, EL(res[r], displs[invr[b]]), R[r], (size_t)rc[invr[b]]);
        else red(c, EL(tmp[r], displs[invr[b]]), EL(res[r], displs[invr[b]]), (size_t)rc[invr[b]]);
      }
    }
    mask <<= 1; inv >>= 1; bfm >>= 1;
  }
  free(displs); free(invr); free_ranks(tmp, P); free_ranks(res, P);
}

/* reduce_scatter_bine_block_by_block_any_even, :1176-1298 */
static void rs_bine_bbb_any_even(ctx_t *c, const int *rc, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (P % 2 && P > 1) {
    /* odd P: the reference hangs (no vector) and its
     * partners leave the communicator; MPI_ERR_ARG, as the device path */
    for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG;
    return;
  }
  int *displs = (int *)malloc(sizeof(int) * (size_t)P), count = 0;
  for (int i = 0; i < P; i++) { displs[i] = count; count += rc[i]; }
  char **tmp = alloc_ranks(P, (size_t)count * esz), **res = alloc_ranks(P, (size_t)count * esz);
  for (int r = 0; r < P; r++) memcpy(res[r], S[r], (size_t)count * esz);
  int **btr = (int **)malloc(sizeof(int *) * (size_t)P);
  int *nrr = (int *)calloc((size_t)P, sizeof(int)), *done = (int *)calloc((size_t)P, sizeof(int));
  for (int r = 0; r < P; r++) btr[r] = (int *)malloc(sizeof(int) * (size_t)(P + 1));
  int mask = 1, rstep = log_2(P) - 1;
  while (mask < P) {
    int lastst = (mask << 1) >= P;
    for (int r = 0; r < P; r++) {
      int partner = nb_partner(r, mask, P);
      nrr[r] = 0;
      for (int block = 1; block < P; block++) {
        int k = 31 - __builtin_clz(orc_get_nu((uint32_t)block, (uint32_t)P));
        if (k != rstep) continue;
        int bts, brv;
        if (r % 2 == 0) { bts = mod(block + r, P); brv = mod(partner - block, P); }
        else { bts = mod(r - block, P); brv = mod(block + partner, P); }
        if (bts != r) b_send(&c->b, r, partner, EL(res[r], displs[bts]), (size_t)rc[bts] * esz);
        if (brv != partner) {
          btr[r][nrr[r]++] = brv;
          if (lastst) { b_recv(&c->b, r, partner, R[r], (size_t)rc[brv] * esz); done[r] = 1; }
          else b_recv(&c->b, r, partner, EL(tmp[r], displs[brv]), (size_t)rc[brv] * esz);
        }
      }
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++)
      for (int i = 0; i < nrr[r]; i++) {
        int b = btr[r][i];
        if (lastst) red(c, EL(res[r], displs[b]), R[r], (size_t)rc[b]);
        else red(c, EL(tmp[r], displs[b]), EL(res[r], displs[b]), (size_t)rc[b]);
      }
    mask <<= 1; rstep--;
  }
  for (int r = 0; r < P; r++)
    if (!done[r] && rc[r]) memcpy(R[r], EL(res[r], displs[r]), (size_t)rc[r] * esz);
  for (int r = 0; r < P; r++) free(btr[r]);
  free(btr); free(nrr); free(done); free(displs); free_ranks(tmp, P); free_ranks(res, P);
}

int orc_reduce_scatter(const char *algo, int P, const int *rcounts, int dtype,
                       int op, const void *const *sbufs, void *const *rbufs,
                       int *rets) {
  if (P < 1 || !orc_dtype_size(dtype)) return -1;
  ctx_t c; memset(&c, 0, sizeof c);
  c.P = P; c.dtype = dtype; c.op = op; c.esz = orc_dtype_size(dtype);
  char **S = (char **)sbufs, **R = (char **)rbufs;
  for (int r = 0; r < P; r++) rets[r] = ORC_OK;
  int known = 1;
  if (!strcmp(algo, "recursivehalving")) rs_recursivehalving(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "recursive_distance_doubling")) rs_recursive_distance_doubling(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "ring")) rs_ring(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "butterfly")) rs_butterfly(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "bine_static")) rs_bine_static(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "bine_send_remap")) rs_bine_remap(&c, rcounts, S, R, rets, 0);
  else if (!strcmp(algo, "bine_permute_remap")) rs_bine_remap(&c, rcounts, S, R, rets, 1);
  else if (!strcmp(algo, "bine_block_by_block")) rs_bine_bbb(&c, rcounts, S, R, rets);
  else if (!strcmp(algo, "bine_block_by_block_any_even")) rs_bine_bbb_any_even(&c, rcounts, S, R, rets);
  else known = 0;
  if (c.dead) for (int r = 0; r < P; r++) if (rets[r] == ORC_OK) rets[r] = c.dead;
  b_free(&c.b);
  return known ? 0 : -1;
}

/* ----------------------------------------------------------------------- */
/* reduce -- libbine_reduce.c                                                */
/* ----------------------------------------------------------------------- */

/* reduce_bine_lat, :16-80 */
static void rd_bine_lat(ctx_t *c, size_t count, int root, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  if (count == 0) return;
  if (!is_pow2(P)) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_SIZE; return; }
  char **tmp = alloc_ranks(P, nb), **acc = alloc_ranks(P, nb);
  char **rb = (char **)malloc(sizeof(char *) * (size_t)P);
  int *quit = (int *)calloc((size_t)P, sizeof(int)), *recv_from = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) { rb[r] = r == root ? R[r] : acc[r]; memcpy(rb[r], S[r], nb); }
  for (int mask = 1; mask < P; mask <<= 1) {                         /* :47-65 */
    for (int r = 0; r < P; r++) {
      recv_from[r] = -1;
      if (quit[r]) continue;
      int vrank = mod(r - root, P);
      int bv = (int)b2nb(vrank);
      int partner = mod(nb2b((uint32_t)(bv ^ ((mask << 1) - 1))) + root, P);
      int ml = (mask << 2) - 1, lsbs = bv & ml;
      int eq = lsbs == 0 || lsbs == ml;
      if (!eq || ((mask << 1) >= P && r != root)) { b_send(&c->b, r, partner, rb[r], nb); quit[r] = 1; }
      else { b_recv(&c->b, r, partner, tmp[r], nb); recv_from[r] = partner; }
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++) if (recv_from[r] >= 0) red(c, tmp[r], rb[r], count);
  }
  free_ranks(tmp, P); free_ranks(acc, P); free(rb); free(quit); free(recv_from);
}

/* reduce_bine_bdw, :83-222 */
static void rd_bine_bdw(ctx_t *c, size_t count, int root, char **S, char **R, int *rets) {
  int P = c->P; size_t esz = c->esz, nb = count * esz;
  if (root != 0) { for (int r = 0; r < P; r++) rets[r] = ORC_ASSERT; return; }   /* :86 */
  int steps = log_2(P);
  if (!is_pow2(P)) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_SIZE; return; }
  int cpr = (int)(count / (size_t)P), rem = (int)(count % (size_t)P);
  char **tmp = alloc_ranks(P, nb), **own = alloc_ranks(P, nb);
  char **res = (char **)malloc(sizeof(char *) * (size_t)P);
  for (int r = 0; r < P; r++) { res[r] = r == root ? R[r] : own[r]; if (nb) memcpy(res[r], S[r], nb); }
  int ns = steps > 0 ? steps : 1;
  int *ri = (int *)calloc((size_t)(P * ns), sizeof(int)), *si = (int *)calloc((size_t)(P * ns), sizeof(int));
  int *rcn = (int *)calloc((size_t)(P * ns), sizeof(int)), *scn = (int *)calloc((size_t)(P * ns), sizeof(int));
#define MN(a, b) ((a) < (b) ? (a) : (b))
  int mask = 1, inv = (int)(1u << ((unsigned)(steps - 1) & 31u)), bfm = (int)~((unsigned)inv - 1u), step = 0;
  while (mask < P) {                                                 /* :128-164 */
    for (int r = 0; r < P; r++) {
      int partner = nb_partner(r, mask, P);
      int sbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)partner) & bfm, sbl = sbf + inv - 1;
      si[r * ns + step] = cpr * sbf + (sbf < rem ? sbf : rem);
      scn[r * ns + step] = cpr * (sbl - sbf + 1) + (MN(sbl, rem) - MN(sbf, rem)) + (sbl < rem ? 1 : 0);
      int rbf = (int)orc_remap_rank((uint32_t)P, (uint32_t)r) & bfm, rbl = rbf + inv - 1;
      ri[r * ns + step] = cpr * rbf + (rbf < rem ? rbf : rem);
      rcn[r * ns + step] = cpr * (rbl - rbf + 1) + (MN(rbl, rem) - MN(rbf, rem)) + (rbl < rem ? 1 : 0);
      b_send(&c->b, r, partner, EL(res[r], si[r * ns + step]), (size_t)scn[r * ns + step] * esz);
      b_recv(&c->b, r, partner, EL(tmp[r], ri[r * ns + step]), (size_t)rcn[r * ns + step] * esz);
    }
    deliver(c, rets);
    for (int r = 0; r < P; r++)
      red(c, EL(tmp[r], ri[r * ns + step]), EL(res[r], ri[r * ns + step]), (size_t)rcn[r * ns + step]);
    mask <<= 1; inv >>= 1; bfm >>= 1; step++;
  }
#undef MN
  mask >>= 1; inv = 1; step = steps - 1;
  int *quit = (int *)calloc((size_t)P, sizeof(int));
  while (mask > 0) {                                                 /* :174-199 */
    for (int r = 0; r < P; r++) {
      if (quit[r]) continue;
      int partner = nb_partner(r, mask, P);
      int rr = (int)orc_remap_rank((uint32_t)P, (uint32_t)r);
      /* 1 << (ffs(0) - 1) is 1 << -1: on the reference's x86 build the count
       * is masked to 31, i.e. bit 31 -- the root never sends */
      unsigned recvmask = rr ? 1u << (__builtin_ffs(rr) - 1) : 0x80000000u;
      if ((unsigned)inv & recvmask) {
        b_send(&c->b, r, partner, EL(res[r], ri[r * ns + step]), (size_t)rcn[r * ns + step] * esz);
        quit[r] = 1;
      } else b_recv(&c->b, r, partner, EL(res[r], si[r * ns + step]), (size_t)scn[r * ns + step] * esz);
    }
    deliver(c, rets);
    mask >>= 1; inv <<= 1; step--;
  }
  free_ranks(tmp, P); free_ranks(own, P); free(res); free(ri); free(si); free(rcn); free(scn); free(quit);
}

int orc_reduce(const char *algo, int P, size_t count, int dtype, int op,
               int root, const void *const *sbufs, void *const *rbufs,
               int *rets) {
  if (P < 1 || !orc_dtype_size(dtype) || root < 0 || root >= P) return -1;
  ctx_t c; memset(&c, 0, sizeof c);
  c.P = P; c.dtype = dtype; c.op = op; c.esz = orc_dtype_size(dtype);
  char **S = (char **)sbufs, **R = (char **)rbufs;
  for (int r = 0; r < P; r++) rets[r] = ORC_OK;
  int known = 1;
  if (!strcmp(algo, "bine_lat")) rd_bine_lat(&c, count, root, S, R, rets);
  else if (!strcmp(algo, "bine_bdw")) rd_bine_bdw(&c, count, root, S, R, rets);
  else known = 0;
  if (c.dead) for (int r = 0; r < P; r++) if (rets[r] == ORC_OK) rets[r] = c.dead;
  b_free(&c.b);
  return known ? 0 : -1;
}

/* ----------------------------------------------------------------------- */
/* allgather -- libbine_allgather.c                                          */
/* ----------------------------------------------------------------------- */
/* R[r] holds P * count elements (pico_core callocs it,
 * pico_core_allgather_utils.c:20).  inpl = MPI_IN_PLACE: S is unused and rank
 * r's block already sits in R[r] where the algorithm expects it.  Each
 * COPY_BUFF_DIFF_DT / copy_buffer with a zero count returns MPI_ERR_UNKNOWN
 * (libbine_utils.h:176-215). */

#define BLK(r, b) EL(R[r], (size_t)(b) * count)

/* copy_buffer_different_dt with equal types, libbine_utils.h:207-228 */
static int cpy(const void *src, void *dst, size_t n, size_t esz) {
  if (n == 0 || !src || !dst) return ORC_ERR_UNKNOWN;
  memmove(dst, src, n * esz);
  return ORC_OK;
}

/* allgather_recursivedoubling, :18-86.  Non-power-of-two P jumps to the error
 * label with err still MPI_SUCCESS (:31-34): nothing happens, success. */
static void ag_recursivedoubling(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (!is_pow2(P)) return;
  for (int r = 0; r < P; r++)
    if (!inpl && (rets[r] = cpy(S[r], BLK(r, r), count, esz))) return;
  int *sbl = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) sbl[r] = r;
  for (int d = 1; d < P; d <<= 1) {
    for (int r = 0; r < P; r++) {
      int remote = r ^ d;
      int rb = r < remote ? sbl[r] + d : sbl[r] - d;
      b_send(&c->b, r, remote, BLK(r, sbl[r]), (size_t)d * count * esz);
      b_recv(&c->b, r, remote, BLK(r, rb), (size_t)d * count * esz);
      if (r > remote) sbl[r] -= d;
    }
    deliver(c, rets);
  }
  free(sbl);
}

/* allgather_k_bruck, radix 2, :88-211 */
static void ag_k_bruck(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  for (int r = 0; r < P; r++) {
    if (!inpl) rets[r] = cpy(S[r], BLK(r, 0), count, esz);
    else if (r != 0) rets[r] = cpy(BLK(r, r), BLK(r, 0), count, esz);
    if (rets[r]) return;
  }
  for (int d = 1; d < P; d *= 2) {                                   /* :158-181 */
    size_t rc = d <= P / 2 ? (size_t)d : (size_t)(d < P - d ? d : P - d);
    for (int r = 0; r < P; r++) {
      b_recv(&c->b, r, (r + d) % P, BLK(r, d), rc * count * esz);
      b_send(&c->b, r, (r - d + P) % P, BLK(r, 0), rc * count * esz);
    }
    deliver(c, rets);
  }
  for (int r = 1; r < P; r++) {                                      /* :185-196 */
    size_t hi = (size_t)(P - r) * count;
    char *t = (char *)malloc(hi * esz);
    memcpy(t, BLK(r, 0), hi * esz);
    memmove(BLK(r, 0), BLK(r, P - r), (size_t)r * count * esz);
    memcpy(BLK(r, r), t, hi * esz);
    free(t);
  }
}

/* allgather_ring, :213-270 */
static void ag_ring(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  for (int r = 0; r < P; r++)
    if (!inpl && (rets[r] = cpy(S[r], BLK(r, r), count, esz))) return;
  for (int i = 0; i < P - 1; i++) {
    for (int r = 0; r < P; r++) {
      b_send(&c->b, r, (r + 1) % P, BLK(r, (r - i + P) % P), count * esz);
      b_recv(&c->b, r, (r - 1 + P) % P, BLK(r, (r - i - 1 + P) % P), count * esz);
    }
    deliver(c, rets);
  }
}

/* allgather_sparbit, :327-408 (tags = block displacement) */
static void ag_sparbit(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  for (int r = 0; r < P; r++)
    if (!inpl && (rets[r] = cpy(S[r], BLK(r, r), count, esz))) return;
  int L = log_2(P), expected = 1;
  uint32_t d = L >= 1 ? 1u << (L - 1) : 0;
  uint32_t last_ignore = (uint32_t)__builtin_ctz((unsigned)P);
  uint32_t ignore = (~((uint32_t)P >> last_ignore) | 1u) << last_ignore;
  for (int i = 0; i < L; i++) {
    int excl = (d & ignore) == d;
    for (int r = 0; r < P; r++) {
      int to = (int)((r + (int)d) % P), from = (int)((r - (int)d + P) % P);
      for (int t = 0; t < expected - excl; t++) {
        int sd = (r - 2 * t * (int)d + P) % P, rd = (r - (2 * t + 1) * (int)d + P) % P;
        b_send_t(&c->b, r, to, BLK(r, sd), count * esz, sd);
        b_recv_t(&c->b, r, from, BLK(r, rd), count * esz, rd);
      }
    }
    deliver(c, rets);
    d >>= 1;
    expected = (expected << 1) - excl;
  }
}

/* get_indexes / get_indexes_aux, libbine_utils.h:142-161 */
static void idx_aux(int rank, int step, int n, int P, int *bm) {
  for (int s = step; s < n; s++) { int p = orc_pi(rank, s, P); bm[p] = 1; idx_aux(p, s + 1, n, P, bm); }
}
static void get_indexes(int rank, int step, int n, int P, int *bm) {
  if (step >= n) return;
  int p = orc_pi(rank, step, P); bm[p] = 1; idx_aux(p, step + 1, n, P, bm);
}

/* allgather_bine_block_by_block, :410-490 (tag = block) */
static void ag_bine_bbb(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  for (int r = 0; r < P; r++)
    if (!inpl && (rets[r] = cpy(S[r], BLK(r, r), count, esz))) return;
  int *sb = (int *)malloc(sizeof(int) * (size_t)P), *rb = (int *)malloc(sizeof(int) * (size_t)P);
  for (int step = steps - 1; step >= 0; step--) {
    for (int r = 0; r < P; r++) {
      int remote = orc_pi(r, step, P);
      memset(sb, 0, sizeof(int) * (size_t)P); memset(rb, 0, sizeof(int) * (size_t)P);
      get_indexes(r, step, steps, P, rb);
      get_indexes(remote, step, steps, P, sb);
      for (int b = 0; b < P; b++) {
        if (sb[b]) b_send_t(&c->b, r, remote, BLK(r, b), count * esz, b);
        if (rb[b]) b_recv_t(&c->b, r, remote, BLK(r, b), count * esz, b);
      }
    }
    deliver(c, rets);
  }
  free(sb); free(rb);
}

/* allgather_bine_block_by_block_any_even, :492-561 (always copies sbuf) */
static void ag_bine_bbb_any_even(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets) {
  int P = c->P; size_t esz = c->esz;
  if (inpl) { for (int r = 0; r < P; r++) rets[r] = ORC_ASSERT; return; }   /* memcpy from MPI_IN_PLACE */
  for (int r = 0; r < P; r++) if (count) memcpy(BLK(r, r), S[r], count * esz);
  int inv = (int)(1u << ((unsigned)(log_2(P) - 1) & 31u)), step = 0;
  while (inv > 0) {
    for (int r = 0; r < P; r++) {
      int d = nb2b((uint32_t)((inv << 1) - 1));
      int partner = r % 2 == 0 ? mod(r + d, P) : mod(r - d, P);
      for (int b = 1; b < P; b++) {
        int k = 31 - __builtin_clz(orc_get_nu((uint32_t)b, (uint32_t)P));
        if (k != step) continue;
        int btr, bts;
        if (r % 2 == 0) { btr = mod(b + r, P); bts = mod(partner - b, P); }
        else { btr = mod(r - b, P); bts = mod(b + partner, P); }
        b_send(&c->b, r, bts != partner ? partner : -1, BLK(r, bts), count * esz);
        b_recv(&c->b, r, btr != r ? partner : -1, BLK(r, btr), count * esz);
      }
    }
    deliver(c, rets);
    inv >>= 1; step++;
  }
}

/* reorder_blocks, libbine_utils.h:438-479: new[i] = old[perm[i]] */
static void reorder(char *buf, size_t bb, const int *perm, int P) {
  char *t = (char *)malloc(bb * (size_t)P);
  memcpy(t, buf, bb * (size_t)P);
  for (int i = 0; i < P; i++) memcpy(buf + (size_t)i * bb, t + (size_t)perm[i] * bb, bb);
  free(t);
}

/* allgather_bine_permute_static (:563-640) and _send_static (:642-723) */
static void ag_bine_static(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets, int permute) {
  int P = c->P; size_t esz = c->esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1 || steps > 8) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  int *perm = (int *)malloc(sizeof(int) * (size_t)P);
  int *st = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps), *rt = (int *)malloc(sizeof(int) * (size_t)P * (size_t)steps);
  orc_static_tables(P, perm, st, rt);
  if (permute) {
    for (int r = 0; r < P; r++)
      if (!inpl && (rets[r] = cpy(S[r], BLK(r, rt[r * steps + steps - 1]), count, esz))) goto out;
  } else {
    for (int r = 0; r < P; r++) {                                    /* :680-696 */
      if (perm[r] != r) {
        int to = -1;
        for (int j = 0; j < P; j++) if (perm[j] == r) { to = j; break; }
        b_send(&c->b, r, to, S[r], count * esz);
        b_recv(&c->b, r, perm[r], BLK(r, perm[r]), count * esz);
      } else if ((rets[r] = cpy(S[r], BLK(r, perm[r]), count, esz))) goto out;
    }
    deliver(c, rets);
  }
  size_t sc = count;
  for (int step = steps - 1; step >= 0; step--) {                    /* :613-626 */
    for (int r = 0; r < P; r++) {
      int remote = orc_pi(r, step, P);
      b_send(&c->b, r, remote, BLK(r, rt[r * steps + step]), sc * esz);
      b_recv(&c->b, r, remote, BLK(r, st[r * steps + step]), sc * esz);
    }
    deliver(c, rets);
    sc *= 2;
  }
  if (permute) for (int r = 0; r < P; r++) reorder(R[r], count * esz, perm, P);
out:
  free(perm); free(st); free(rt);
}

/* get_sender_rec, libbine_utils.h:585-594: x with remap_rank(x) == rank */
static int sender_rec(int P, int rank) {
  int x = rank;
  for (;;) { int m = (int)orc_remap_rank((uint32_t)P, (uint32_t)x); if (m == rank) return x; x = m; }
}

/* allgather_bine_permute_remap (:725-809) and _send_remap (:811-890) */
static void ag_bine_remap(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets, int permute) {
  int P = c->P; size_t esz = c->esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1 || steps > 8) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  int *remap = (int *)malloc(sizeof(int) * (size_t)P), *sbl = (int *)malloc(sizeof(int) * (size_t)P);
  for (int r = 0; r < P; r++) remap[r] = (int)orc_remap_rank((uint32_t)P, (uint32_t)r);
  if (permute) {
    for (int r = 0; r < P; r++)
      if (!inpl && (rets[r] = cpy(S[r], BLK(r, remap[r]), count, esz))) goto out;
  } else {
    for (int r = 0; r < P; r++) {                                    /* :840-853 */
      if (remap[r] != r) {
        b_send(&c->b, r, sender_rec(P, r), S[r], count * esz);
        b_recv(&c->b, r, remap[r], BLK(r, remap[r]), count * esz);
      } else if ((rets[r] = cpy(S[r], BLK(r, remap[r]), count, esz))) goto out;
    }
    deliver(c, rets);
  }
  for (int r = 0; r < P; r++) sbl[r] = remap[r];
  int d = 1;
  for (int step = steps - 1; step >= 0; step--) {                    /* :776-795 */
    for (int r = 0; r < P; r++) {
      int remote = orc_pi(r, step, P), vr = remap[r], vrem = remap[remote];
      int rb = vr < vrem ? sbl[r] + d : sbl[r] - d;
      b_send(&c->b, r, remote, BLK(r, sbl[r]), (size_t)d * count * esz);
      b_recv(&c->b, r, remote, BLK(r, rb), (size_t)d * count * esz);
      if (!(vr < vrem)) sbl[r] -= d;
    }
    deliver(c, rets);
    d <<= 1;
  }
  if (permute) for (int r = 0; r < P; r++) reorder(R[r], count * esz, remap, P);
out:
  free(remap); free(sbl);
}

/* allgather_bine_2_blocks (:892-997, extra wrap-around message with tag 1)
 * and _2_blocks_dtype (:999-1106, one message packed by MPI_Type_indexed:
 * wrapped head first, then the main run) */
static void ag_bine_2_blocks(ctx_t *c, size_t count, char **S, char **R, int inpl, int *rets, int dtype_variant) {
  int P = c->P; size_t esz = c->esz;
  int steps = log_2(P);
  if (!is_pow2(P) || steps < 1) { for (int r = 0; r < P; r++) rets[r] = ORC_ERR_ARG; return; }
  for (int r = 0; r < P; r++)
    if (!inpl && (rets[r] = cpy(S[r], BLK(r, r), count, esz))) return;
  int *first = (int *)malloc(sizeof(int) * (size_t)P);
  int *ri = (int *)malloc(sizeof(int) * (size_t)P), *xr = (int *)malloc(sizeof(int) * (size_t)P);
  char **stage = alloc_ranks(P, (size_t)P * count * esz);
  for (int r = 0; r < P; r++) first[r] = r;
  int mask = 1;
  for (int step = 0; step < steps; step++) {
    for (int r = 0; r < P; r++) {
      int remote = orc_pi(r, step, P), si = first[r], rix;
      if ((step & 1) == (r & 1)) rix = (si + mask + P) % P;
      else { rix = (si - mask + P) % P; first[r] = rix; }
      int xrv = rix + mask > P ? rix + mask - P : 0, xsd = si + mask > P ? si + mask - P : 0;
      int rcn = mask - xrv, scn = mask - xsd;
      ri[r] = rix; xr[r] = xrv;
      if (!dtype_variant) {
        if (xrv) b_recv_t(&c->b, r, remote, BLK(r, 0), (size_t)xrv * count * esz, 1);
        if (xsd) b_send_t(&c->b, r, remote, BLK(r, 0), (size_t)xsd * count * esz, 1);
        b_send(&c->b, r, remote, BLK(r, si), (size_t)scn * count * esz);
        b_recv(&c->b, r, remote, BLK(r, rix), (size_t)rcn * count * esz);
      } else {
        char *pk = (char *)malloc((size_t)mask * count * esz + 1);
        memcpy(pk, BLK(r, 0), (size_t)xsd * count * esz);
        memcpy(pk + (size_t)xsd * count * esz, BLK(r, si), (size_t)scn * count * esz);
        b_send(&c->b, r, remote, pk, (size_t)mask * count * esz);
        free(pk);
        b_recv(&c->b, r, remote, stage[r], (size_t)mask * count * esz);
      }
    }
    deliver(c, rets);
    if (dtype_variant)
      for (int r = 0; r < P; r++) {
        memcpy(BLK(r, 0), stage[r], (size_t)xr[r] * count * esz);
        memcpy(BLK(r, ri[r]), stage[r] + (size_t)xr[r] * count * esz, (size_t)(mask - xr[r]) * count * esz);
      }
    mask <<= 1;
  }
  free(first); free(ri); free(xr); free_ranks(stage, P);
}
#undef BLK

int orc_allgather(const char *algo, int P, size_t count, int dtype, int in_place,
                  const void *const *sbufs, void *const *rbufs, int *rets) {
  if (P < 1 || !orc_dtype_size(dtype)) return -1;
  ctx_t c; memset(&c, 0, sizeof c);
  c.P = P; c.dtype = dtype; c.esz = orc_dtype_size(dtype);
  char **S = (char **)sbufs, **R = (char **)rbufs;
  for (int r = 0; r < P; r++) rets[r] = ORC_OK;
  int known = 1, ip = in_place != 0;
  if (!strcmp(algo, "recursivedoubling")) ag_recursivedoubling(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "k_bruck")) ag_k_bruck(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "ring")) ag_ring(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "sparbit")) ag_sparbit(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "bine_block_by_block")) ag_bine_bbb(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "bine_block_by_block_any_even")) ag_bine_bbb_any_even(&c, count, S, R, ip, rets);
  else if (!strcmp(algo, "bine_permute_static")) ag_bine_static(&c, count, S, R, ip, rets, 1);
  else if (!strcmp(algo, "bine_send_static")) ag_bine_static(&c, count, S, R, ip, rets, 0);
  else if (!strcmp(algo, "bine_permute_remap")) ag_bine_remap(&c, count, S, R, ip, rets, 1);
  else if (!strcmp(algo, "bine_send_remap")) ag_bine_remap(&c, count, S, R, ip, rets, 0);
  else if (!strcmp(algo, "bine_2_blocks")) ag_bine_2_blocks(&c, count, S, R, ip, rets, 0);
  else if (!strcmp(algo, "bine_2_blocks_dtype")) ag_bine_2_blocks(&c, count, S, R, ip, rets, 1);
  else known = 0;
  if (c.dead) for (int r = 0; r < P; r++) if (rets[r] == ORC_OK) rets[r] = c.dead;
  b_free(&c.b);
  return known ? 0 : -1;
}
