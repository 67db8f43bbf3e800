// kernels.hip -- CDNA4 (gfx950) kernels of libbine_amd.so.
//
//  * k_reduce: the element-wise reduction that replaces MPI_Reduce_local at all
//    32 call sites of libbine's reduce family (e.g. libbine_allreduce.c:888):
//    out[i] = b[i] (op) a[i], out may alias b.  HBM-bound streaming kernel:
//    16 B per lane per access (global_load_dwordx4), U independent 16-B vectors
//    per lane in flight, one tile of 256 x U vectors per workgroup (no grid
//    cap below 16,384 workgroups, no grid-stride loop: measured faster on
//    MI355X, profiles/r1_explore.txt).  No LDS: every byte is touched once, so
//    staging through LDS would only add instructions.  Arithmetic follows
//    MPICH 3.3.2 exactly (inout (op) in, no FMA contraction, no denormal
//    flushing, integer wrap).
//  * k_copy: the device form of libbine's copy_buffer (libbine_utils.h:176-190,
//    e.g. the sbuf -> rbuf copy of allreduce_bine_bdw_remap at
//    libbine_allreduce.c:849-852 -- the whole P = 1 allreduce).  16-B vectors,
//    8 per lane in flight, non-temporal loads AND stores: 83 us for 256 MiB
//    (6.44 TB/s of read + write) vs 98.6 us for hipMemcpyAsync D2D
//    (tools/copy_variants.hip, profiles/r2_copy_variants.txt).
//  * k_fill_pico: pico_core's rand_r() input distributions
//    (pico_core_utils.c:902-923) generated in parallel by LCG jump-ahead,
//    bit-identical to the sequential host generator.
//  * k_checksum: order-independent 64-bit digest for size-independent parity
//    checks at full sizes; per-lane partial sums reduced with wave64 shuffles,
//    then through LDS, then one 64-bit atomic per workgroup.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "bine_internal.h"

// This file is compiled twice (Makefile): BINE_OPSET 0 -> kernels.o, the
// arithmetic ops SUM / PROD / MAX / MIN and every other kernel; BINE_OPSET 1
// -> kernels_logic.o, the reduction kernels' instantiations for the logical
// and bitwise ops only (launch_*_logic, reached from the opset-0 entry
// points).  Two translation units compile in parallel.
#ifndef BINE_OPSET
#define BINE_OPSET 0
#endif
#if BINE_OPSET == 0
#define BINE_FN(name) name
#else
#define BINE_FN(name) name##_logic
#endif

namespace bine {

// ----------------------------------------------------------------------------
// element-wise reduction
// ----------------------------------------------------------------------------

template <typename T>
using uint_of = std::conditional_t<sizeof(T) == 1, uint8_t,
                std::conditional_t<sizeof(T) == 2, uint16_t,
                std::conditional_t<sizeof(T) == 4, uint32_t, uint64_t>>>;

// MPI's (value, index) pair types, C layout.  The padding of the C structs is
// spelled out as members, so that a pair passed and returned by value keeps
// the inout operand's padding bytes (implicit padding is unspecified after a
// copy -- measured: garbage in the padding of returned {double; int} pairs).
template <typename V>
struct Pair {
  V v;
  int i;
};
template <>
struct Pair<double> {
  double v;
  int i, pad_;
};
template <>
struct Pair<long> {
  long v;
  int i, pad_;
};
template <>
struct Pair<short> {
  short v, pad_;
  int i;
};
static_assert(sizeof(Pair<double>) == 16 && sizeof(Pair<long>) == 16 && sizeof(Pair<short>) == 8 &&
                  sizeof(Pair<float>) == 8 && sizeof(Pair<int>) == 8 && offsetof(Pair<short>, i) == 4,
              "MPI pair layouts");
template <typename T>
struct is_pair : std::false_type {};
template <typename V>
struct is_pair<Pair<V>> : std::true_type {};

// C99 complex {re; im} (MPI_C_FLOAT_COMPLEX / MPI_C_DOUBLE_COMPLEX)
template <typename V>
struct Cplx {
  V re, im;
};
template <typename T>
struct is_cplx : std::false_type {};
template <typename V>
struct is_cplx<Cplx<V>> : std::true_type {};

// MPICH's MPIR_OP_TYPE_REDUCE_CASE: a = inout, b = in, a = OP(a, b)
template <typename T, int OP>
__device__ __forceinline__ T apply(T io, T in) {
  if constexpr (is_cplx<T>::value) {
    // MPICH's MPIR_LSUM / MPIR_LPROD on float/double _Complex: component-wise
    // sum; for finite operands the product is (a.re b.re - a.im b.im) +
    // (a.re b.im + a.im b.re) i (a = inout; no FMA: -ffp-contract=off)
    if constexpr (OP == BINE_SUM) {
      io.re = io.re + in.re;
      io.im = io.im + in.im;
    } else {
      static_assert(OP == BINE_PROD, "complex types: SUM / PROD only");
      const auto re = io.re * in.re - io.im * in.im;
      const auto im = io.re * in.im + io.im * in.re;
      io.re = re;
      io.im = im;
    }
    return io;
  } else if constexpr (OP == BINE_SUM) {
    if constexpr (std::is_integral_v<T>) return (T)((uint_of<T>)io + (uint_of<T>)in);
    else return io + in;
  } else if constexpr (OP == BINE_PROD) {
    if constexpr (std::is_integral_v<T>) return (T)((uint_of<T>)io * (uint_of<T>)in);
    else return io * in;
  } else if constexpr (OP == BINE_MAX) {
    return io > in ? io : in;
  } else if constexpr (OP == BINE_MIN) {
    return io < in ? io : in;
  } else if constexpr (OP == BINE_LAND) {  // MPIR_LLAND: C truthiness (-0.0 false, NaN true), 0 / 1
    return (T)(io != (T)0 && in != (T)0);
  } else if constexpr (OP == BINE_LOR) {
    return (T)(io != (T)0 || in != (T)0);
  } else if constexpr (OP == BINE_LXOR) {
    return (T)((io != (T)0) != (in != (T)0));
  } else if constexpr (OP == BINE_BAND) {
    return (T)(io & in);
  } else if constexpr (OP == BINE_BOR) {
    return (T)(io | in);
  } else if constexpr (OP == BINE_MAXLOC || OP == BINE_MINLOC) {
    // MPICH opmaxloc.c / opminloc.c (a = inout, b = in): equal values keep
    // the smaller index; otherwise a strictly larger (smaller) value of `in`
    // replaces the pair -- field by field, so io's padding bytes stay
    if (io.v == in.v) io.i = io.i < in.i ? io.i : in.i;
    else if (OP == BINE_MAXLOC ? io.v < in.v : io.v > in.v) {
      io.v = in.v;
      io.i = in.i;
    }
    return io;
  } else {
    static_assert(OP == BINE_BXOR, "unknown op");
    return (T)(io ^ in);
  }
}

// Which element types each op is instantiated for.  The bitwise ops act on
// bits alone, so every integer type runs them as bytes (canon_dtype below);
// the logical ops depend only on whether an element is zero, so signed
// integers run them as the unsigned type of their width.  The four
// arithmetic ops exist for every type.
template <typename T>
constexpr bool kLogicT = std::is_unsigned_v<T> || std::is_floating_point_v<T>;
template <typename T>
constexpr bool kBitsT = std::is_same_v<T, uint8_t>;
template <typename T>
constexpr bool kPairT = is_pair<T>::value;
template <typename T>
constexpr bool kCplxT = is_cplx<T>::value;

// BINE_OP_SWITCH(T, CALL): `return CALL(OP)` for the op in variable `op`,
// only for the (T, OP) pairs instantiated; hipErrorInvalidValue otherwise
#if BINE_OPSET == 0
#define BINE_OP_SWITCH(T, CALL)                                      \
  switch (op) {                                                      \
    case BINE_SUM: return CALL(BINE_SUM);                            \
    case BINE_PROD: return CALL(BINE_PROD);                          \
    case BINE_MAX: return CALL(BINE_MAX);                            \
    case BINE_MIN: return CALL(BINE_MIN);                            \
    default: break;                                                  \
  }                                                                  \
  return hipErrorInvalidValue;
#else
#define BINE_OP_SWITCH(T, CALL)                                      \
  switch (op) {                                                      \
    case BINE_SUM: if constexpr (kCplxT<T>) return CALL(BINE_SUM); break;   \
    case BINE_PROD: if constexpr (kCplxT<T>) return CALL(BINE_PROD); break; \
    case BINE_LAND: if constexpr (kLogicT<T>) return CALL(BINE_LAND); break; \
    case BINE_LOR: if constexpr (kLogicT<T>) return CALL(BINE_LOR); break;   \
    case BINE_LXOR: if constexpr (kLogicT<T>) return CALL(BINE_LXOR); break; \
    case BINE_BAND: if constexpr (kBitsT<T>) return CALL(BINE_BAND); break;  \
    case BINE_BOR: if constexpr (kBitsT<T>) return CALL(BINE_BOR); break;    \
    case BINE_BXOR: if constexpr (kBitsT<T>) return CALL(BINE_BXOR); break;  \
    case BINE_MAXLOC: if constexpr (kPairT<T>) return CALL(BINE_MAXLOC); break; \
    case BINE_MINLOC: if constexpr (kPairT<T>) return CALL(BINE_MINLOC); break; \
    default: break;                                                  \
  }                                                                  \
  return hipErrorInvalidValue;
#endif

// the (type, op) pairs the opset-1 compilation holds: the logical / bitwise /
// loc ops, and the pair and complex types
[[maybe_unused]] static bool ext_op(int dtype, int op) {
  return (op >= BINE_LAND && op < BINE_NUM_OPS) || (dtype >= BINE_FLOAT_INT && dtype < BINE_NUM_DTYPES);
}

// the element type an op runs on (see kLogicT / kBitsT); *scale = elements
// of the run type per element of `dtype`; -1: the op is not defined on the
// type (bitwise ops on float / double: MPICH's MPI_ERR_OP)
static int canon_dtype(int dtype, int op, size_t *scale) {
  *scale = 1;
  if (!bine_op_valid(dtype, op)) return -1;
  if (op == BINE_BAND || op == BINE_BOR || op == BINE_BXOR) {
    *scale = bine_dtype_size(dtype);
    return BINE_UINT8;
  }
  if (op == BINE_LAND || op == BINE_LOR || op == BINE_LXOR) {
    switch (dtype) {
      case BINE_INT8: return BINE_UINT8;
      case BINE_INT16: return BINE_UINT16;
      case BINE_INT32: return BINE_UINT32;
      case BINE_INT64: return BINE_UINT64;
      default: return dtype;
    }
  }
  return dtype;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <typename T, int OP>
__device__ __forceinline__ u32x4_t apply16(u32x4_t vb, u32x4_t va) {
  constexpr int N = 16 / (int)sizeof(T);
  T b[N], a[N];
  __builtin_memcpy(b, &vb, 16);
  __builtin_memcpy(a, &va, 16);
#pragma unroll
  for (int i = 0; i < N; i++) b[i] = apply<T, OP>(b[i], a[i]);
  u32x4_t r;
  __builtin_memcpy(&r, b, 16);
  return r;
}

constexpr int kBlock = 256;
using u32x4 = u32x4_t;  // one global_load/store_dwordx4 per lane

// Elements [0, head) and [head + 16/sizeof(T) * nvec, n) are done scalar by
// block 0; the 16-B aligned middle is vectorized.  NT is a cache-policy mask:
// bit 0 = non-temporal loads of `a` (the received operand, read exactly once),
// bit 1 = of `b`, bit 2 = non-temporal stores of `out`.
template <int NTBIT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NTBIT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <typename T, int OP, int U, int NT>
__global__ __launch_bounds__(kBlock) void k_reduce(const T *__restrict__ a, const T *b, T *out,
                                                   size_t head, size_t nvec, size_t n) {
  constexpr size_t V = 16 / sizeof(T);
  if (blockIdx.x == 0) {
    for (size_t i = threadIdx.x; i < head; i += kBlock) out[i] = apply<T, OP>(b[i], a[i]);
    for (size_t i = head + nvec * V + threadIdx.x; i < n; i += kBlock) out[i] = apply<T, OP>(b[i], a[i]);
  }
  const u32x4 *va = reinterpret_cast<const u32x4 *>(a + head);
  const u32x4 *vb = reinterpret_cast<const u32x4 *>(b + head);
  u32x4 *vo = reinterpret_cast<u32x4 *>(out + head);
  const size_t tile = (size_t)kBlock * U;
  const size_t stride = (size_t)gridDim.x * tile;
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  // full tiles: no bounds checks, U loads of each operand in flight per lane
  for (; base + (U - 1) * (size_t)kBlock < nvec; base += stride) {
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      x[u] = ld<NT & 1>(va + base + (size_t)u * kBlock);
      y[u] = ld<NT & 2>(vb + base + (size_t)u * kBlock);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 r = apply16<T, OP>(y[u], x[u]);
      if constexpr (NT & 4) __builtin_nontemporal_store(r, vo + base + (size_t)u * kBlock);
      else vo[base + (size_t)u * kBlock] = r;
    }
  }
  // last partial tile
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + (size_t)u * kBlock;
    if (i < nvec) vo[i] = apply16<T, OP>(vb[i], va[i]);
  }
}

// dispatch -----------------------------------------------------------------

// Defaults measured on MI355X (profiles/r1_explore.txt, C2 fp32 SUM 64 MiB):
// 4 vectors per lane, one tile per workgroup (no grid cap below 16384
// workgroups), non-temporal loads of the once-read operand.
constexpr int kDefaultUnroll = 4, kDefaultMaxBlocks = 16384, kDefaultNT = 1;
static int g_unroll = 0, g_maxblocks = 0, g_nt = kDefaultNT;

[[maybe_unused]] static void read_tuning() {
  if (g_unroll) return;
  const char *u = getenv("BINE_REDUCE_UNROLL");
  const char *m = getenv("BINE_REDUCE_MAXBLOCKS");
  const char *t = getenv("BINE_REDUCE_NT");
  int uu = u ? atoi(u) : 4;
  g_unroll = (uu == 1 || uu == 2 || uu == 4 || uu == 8) ? uu : 4;
  g_maxblocks = m ? atoi(m) : 0;
  g_nt = t ? atoi(t) : kDefaultNT;
}

template <typename T, int OP, int U, int NT>
static hipError_t run_reduce(const T *a, const T *b, T *out, size_t n, hipStream_t st) {
  constexpr size_t V = 16 / sizeof(T);
  const uintptr_t ao = (uintptr_t)a, bo = (uintptr_t)b, oo = (uintptr_t)out;
  size_t head, nvec;
  if (((ao ^ oo) & 15) == 0 && ((bo ^ oo) & 15) == 0 && (oo % sizeof(T)) == 0) {
    head = ((16 - (oo & 15)) & 15) / sizeof(T);
    if (head > n) head = n;
    nvec = (n - head) / V;
  } else {  // operands not co-aligned mod 16 B (small runs only, see reduce_t)
    head = n;
    nvec = 0;
  }
  int blocks;
  if (nvec == 0) blocks = 1;
  else {
    const size_t tiles = (nvec + (size_t)kBlock * U - 1) / ((size_t)kBlock * U);
    const int maxb = g_maxblocks > 0 ? g_maxblocks : kDefaultMaxBlocks;
    blocks = (int)(tiles < (size_t)maxb ? tiles : (size_t)maxb);
  }
  hipLaunchKernelGGL((k_reduce<T, OP, U, NT>), dim3(blocks), dim3(kBlock), 0, st, a, b, out, head, nvec, n);
  return hipGetLastError();
}

// scalar grid-stride kernel for operands that are not co-aligned mod 16 bytes
template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(const T *__restrict__ a, const T *b, T *out,
                                                          size_t n) {
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    out[i] = apply<T, OP>(b[i], a[i]);
}

template <typename T, int OP>
static hipError_t reduce_t(const void *a, const void *b, void *out, size_t n, hipStream_t st) {
  const T *pa = (const T *)a, *pb = (const T *)b;
  T *po = (T *)out;
  const uintptr_t ao = (uintptr_t)a, bo = (uintptr_t)b, oo = (uintptr_t)out;
  if ((((ao ^ oo) & 15) != 0 || ((bo ^ oo) & 15) != 0) && n > 4096) {
    size_t blocks = (n + kBlock * 4 - 1) / (kBlock * 4);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL((k_reduce_scalar<T, OP>), dim3((unsigned)blocks), dim3(kBlock), 0, st, pa, pb, po, n);
    return hipGetLastError();
  }
  if constexpr (std::is_same_v<T, float> && OP == BINE_SUM) {
    // tuning variants (bine_set_reduce_tuning / BINE_REDUCE_*) for the headline dtype
#define NTSW(U)                                                               \
    switch (g_nt) {                                                           \
      case 0: return run_reduce<T, OP, U, 0>(pa, pb, po, n, st);              \
      case 2: return run_reduce<T, OP, U, 2>(pa, pb, po, n, st);              \
      case 3: return run_reduce<T, OP, U, 3>(pa, pb, po, n, st);              \
      case 4: return run_reduce<T, OP, U, 4>(pa, pb, po, n, st);              \
      case 5: return run_reduce<T, OP, U, 5>(pa, pb, po, n, st);              \
      case 7: return run_reduce<T, OP, U, 7>(pa, pb, po, n, st);              \
      default: return run_reduce<T, OP, U, 1>(pa, pb, po, n, st);             \
    }
    switch (g_unroll) {
      case 1: NTSW(1)
      case 2: NTSW(2)
      case 8: NTSW(8)
      default: NTSW(4)
    }
#undef NTSW
  }
  return run_reduce<T, OP, kDefaultUnroll, kDefaultNT>(pa, pb, po, n, st);
}

template <typename T>
static hipError_t reduce_op(const void *a, const void *b, void *out, size_t n, int op, hipStream_t st) {
#define CALL(OP) reduce_t<T, OP>(a, b, out, n, st)
  BINE_OP_SWITCH(T, CALL)
#undef CALL
}

int BINE_FN(launch_reduce)(const void *a, const void *b, void *out, size_t count, int dtype, int op, void *stream) {
  if (count == 0) return BINE_SUCCESS;
#if BINE_OPSET == 0
  if (ext_op(dtype, op)) return launch_reduce_logic(a, b, out, count, dtype, op, stream);
#endif
  size_t scale;
  dtype = canon_dtype(dtype, op, &scale);
  if (dtype < 0) return BINE_ERR_ARG;
  count *= scale;
  read_tuning();
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case BINE_INT8: e = reduce_op<int8_t>(a, b, out, count, op, st); break;
    case BINE_UINT8: e = reduce_op<uint8_t>(a, b, out, count, op, st); break;
    case BINE_INT16: e = reduce_op<int16_t>(a, b, out, count, op, st); break;
    case BINE_UINT16: e = reduce_op<uint16_t>(a, b, out, count, op, st); break;
    case BINE_INT32: e = reduce_op<int32_t>(a, b, out, count, op, st); break;
    case BINE_UINT32: e = reduce_op<uint32_t>(a, b, out, count, op, st); break;
    case BINE_INT64: e = reduce_op<int64_t>(a, b, out, count, op, st); break;
    case BINE_UINT64: e = reduce_op<uint64_t>(a, b, out, count, op, st); break;
    case BINE_FLOAT: e = reduce_op<float>(a, b, out, count, op, st); break;
    case BINE_DOUBLE: e = reduce_op<double>(a, b, out, count, op, st); break;
#if BINE_OPSET == 1
    case BINE_FLOAT_INT: e = reduce_op<Pair<float>>(a, b, out, count, op, st); break;
    case BINE_DOUBLE_INT: e = reduce_op<Pair<double>>(a, b, out, count, op, st); break;
    case BINE_LONG_INT: e = reduce_op<Pair<long>>(a, b, out, count, op, st); break;
    case BINE_2INT: e = reduce_op<Pair<int>>(a, b, out, count, op, st); break;
    case BINE_SHORT_INT: e = reduce_op<Pair<short>>(a, b, out, count, op, st); break;
    case BINE_C_FLOAT_COMPLEX: e = reduce_op<Cplx<float>>(a, b, out, count, op, st); break;
    case BINE_C_DOUBLE_COMPLEX: e = reduce_op<Cplx<double>>(a, b, out, count, op, st); break;
#endif
    default: return BINE_ERR_UNSUPPORTED;
  }
  return e == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

#if BINE_OPSET == 0
// ----------------------------------------------------------------------------
// device copy (copy_buffer): one tile of kBlock * kCopyU 16-B vectors per
// workgroup, loads issued before stores, both non-temporal (the copied bytes
// are not re-read by this launch).  Bytes before the first 16-B boundary of
// `dst` and after the last full vector go byte-wise through workgroup 0.
constexpr int kCopyU = 8;

__global__ __launch_bounds__(kBlock) void k_copy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                 size_t head, size_t nvec, size_t n) {
  if (blockIdx.x == 0) {
    for (size_t i = threadIdx.x; i < head; i += kBlock) dst[i] = src[i];
    for (size_t i = head + nvec * 16 + threadIdx.x; i < n; i += kBlock) dst[i] = src[i];
  }
  const u32x4 *vs = reinterpret_cast<const u32x4 *>(src + head);
  u32x4 *vd = reinterpret_cast<u32x4 *>(dst + head);
  const size_t base = (size_t)blockIdx.x * kBlock * kCopyU + threadIdx.x;
  if (base + (kCopyU - 1) * (size_t)kBlock < nvec) {
    u32x4 x[kCopyU];
#pragma unroll
    for (int u = 0; u < kCopyU; u++) x[u] = __builtin_nontemporal_load(vs + base + (size_t)u * kBlock);
#pragma unroll
    for (int u = 0; u < kCopyU; u++) __builtin_nontemporal_store(x[u], vd + base + (size_t)u * kBlock);
  } else {
#pragma unroll
    for (int u = 0; u < kCopyU; u++) {
      const size_t i = base + (size_t)u * kBlock;
      if (i < nvec) vd[i] = vs[i];
    }
  }
}

int launch_copy(void *dst, const void *src, size_t bytes, void *stream) {
  if (bytes == 0 || dst == src) return BINE_SUCCESS;
  hipStream_t st = (hipStream_t)stream;
  const uintptr_t so = (uintptr_t)src, dO = (uintptr_t)dst;
  if ((so ^ dO) & 15) {
    // not co-aligned mod 16 B (never the case for the plans' element offsets of
    // 16-B aligned buffers): the runtime's device copy
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
  }
  size_t head = (16 - (dO & 15)) & 15;
  if (head > bytes) head = bytes;
  const size_t nvec = (bytes - head) / 16;
  const size_t tiles = (nvec + (size_t)kBlock * kCopyU - 1) / ((size_t)kBlock * kCopyU);
  const unsigned blocks = (unsigned)(tiles ? tiles : 1);
  hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(kBlock), 0, st, (const uint8_t *)src, (uint8_t *)dst, head, nvec,
                     bytes);
  return hipGetLastError() == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}


#endif  // BINE_OPSET == 0

// ----------------------------------------------------------------------------
// batched reduction: up to kMaxBatch independent windows in one launch (the
// P-1 per-instance chunk reductions of a multi-tree round).  The grid is the
// concatenation of every window's tiles; a workgroup finds its window by a
// scan over at most 8 tile offsets.  Windows must be co-aligned mod 16 B
// (the caller falls back to one launch per window otherwise).

struct BatchWin {
  const void *a, *b;
  void *out;
  uint64_t head, nvec, n, tile0;
};
struct Batch {
  int nwin;
  BatchWin w[kMaxBatch];
};

template <typename T, int OP, int U, int NT>
__global__ __launch_bounds__(kBlock) void k_reduce_batch(Batch bt) {
  constexpr size_t V = 16 / sizeof(T);
  const uint64_t t = blockIdx.x;
  int k = 0;
  while (k + 1 < bt.nwin && t >= bt.w[k + 1].tile0) k++;
  const BatchWin &w = bt.w[k];
  const T *a = (const T *)w.a, *b = (const T *)w.b;
  T *out = (T *)w.out;
  if (t == w.tile0) {  // head and tail of this window
    for (size_t i = threadIdx.x; i < w.head; i += kBlock) out[i] = apply<T, OP>(b[i], a[i]);
    for (size_t i = w.head + w.nvec * V + threadIdx.x; i < w.n; i += kBlock) out[i] = apply<T, OP>(b[i], a[i]);
  }
  const u32x4 *va = reinterpret_cast<const u32x4 *>(a + w.head);
  const u32x4 *vb = reinterpret_cast<const u32x4 *>(b + w.head);
  u32x4 *vo = reinterpret_cast<u32x4 *>(out + w.head);
  const size_t base = (size_t)(t - w.tile0) * kBlock * U + threadIdx.x;
  if (base + (U - 1) * (size_t)kBlock < w.nvec) {
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      x[u] = ld<NT & 1>(va + base + (size_t)u * kBlock);
      y[u] = ld<NT & 2>(vb + base + (size_t)u * kBlock);
    }
#pragma unroll
    for (int u = 0; u < U; u++) vo[base + (size_t)u * kBlock] = apply16<T, OP>(y[u], x[u]);
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * kBlock;
      if (i < w.nvec) vo[i] = apply16<T, OP>(vb[i], va[i]);
    }
  }
}

template <typename T, int OP>
static hipError_t batch_t(int n, const void *const *a, const void *const *b, void *const *out,
                          const size_t *count, hipStream_t st) {
  constexpr int U = kDefaultUnroll;
  constexpr size_t V = 16 / sizeof(T);
  Batch bt;
  bt.nwin = n;
  uint64_t tiles = 0;
  for (int k = 0; k < n; k++) {
    const uintptr_t ao = (uintptr_t)a[k], bo = (uintptr_t)b[k], oo = (uintptr_t)out[k];
    if (((ao ^ oo) & 15) || ((bo ^ oo) & 15) || (oo % sizeof(T))) return hipErrorInvalidValue;
    BatchWin &w = bt.w[k];
    w.a = a[k];
    w.b = b[k];
    w.out = out[k];
    w.n = count[k];
    w.head = std::min<uint64_t>(((16 - (oo & 15)) & 15) / sizeof(T), w.n);
    w.nvec = (w.n - w.head) / V;
    w.tile0 = tiles;
    tiles += std::max<uint64_t>(1, (w.nvec + (uint64_t)kBlock * U - 1) / ((uint64_t)kBlock * U));
  }
  hipLaunchKernelGGL((k_reduce_batch<T, OP, U, kDefaultNT>), dim3((unsigned)tiles), dim3(kBlock), 0, st, bt);
  return hipGetLastError();
}

template <typename T>
static hipError_t batch_op(int n, const void *const *a, const void *const *b, void *const *out, const size_t *c,
                           int op, hipStream_t st) {
#define CALL(OP) batch_t<T, OP>(n, a, b, out, c, st)
  BINE_OP_SWITCH(T, CALL)
#undef CALL
}

int BINE_FN(launch_reduce_batch)(int n, const void *const *a, const void *const *b, void *const *out,
                                 const size_t *count_in, int dtype, int op, void *stream) {
  if (n < 1 || n > kMaxBatch) return BINE_ERR_ARG;
#if BINE_OPSET == 0
  if (ext_op(dtype, op)) return launch_reduce_batch_logic(n, a, b, out, count_in, dtype, op, stream);
#endif
  size_t scale;
  dtype = canon_dtype(dtype, op, &scale);
  if (dtype < 0) return BINE_ERR_ARG;
  size_t count[kMaxBatch];
  for (int k = 0; k < n; k++) count[k] = count_in[k] * scale;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case BINE_INT8: e = batch_op<int8_t>(n, a, b, out, count, op, st); break;
    case BINE_UINT8: e = batch_op<uint8_t>(n, a, b, out, count, op, st); break;
    case BINE_INT16: e = batch_op<int16_t>(n, a, b, out, count, op, st); break;
    case BINE_UINT16: e = batch_op<uint16_t>(n, a, b, out, count, op, st); break;
    case BINE_INT32: e = batch_op<int32_t>(n, a, b, out, count, op, st); break;
    case BINE_UINT32: e = batch_op<uint32_t>(n, a, b, out, count, op, st); break;
    case BINE_INT64: e = batch_op<int64_t>(n, a, b, out, count, op, st); break;
    case BINE_UINT64: e = batch_op<uint64_t>(n, a, b, out, count, op, st); break;
    case BINE_FLOAT: e = batch_op<float>(n, a, b, out, count, op, st); break;
    case BINE_DOUBLE: e = batch_op<double>(n, a, b, out, count, op, st); break;
#if BINE_OPSET == 1
    case BINE_FLOAT_INT: e = batch_op<Pair<float>>(n, a, b, out, count, op, st); break;
    case BINE_DOUBLE_INT: e = batch_op<Pair<double>>(n, a, b, out, count, op, st); break;
    case BINE_LONG_INT: e = batch_op<Pair<long>>(n, a, b, out, count, op, st); break;
    case BINE_2INT: e = batch_op<Pair<int>>(n, a, b, out, count, op, st); break;
    case BINE_SHORT_INT: e = batch_op<Pair<short>>(n, a, b, out, count, op, st); break;
    case BINE_C_FLOAT_COMPLEX: e = batch_op<Cplx<float>>(n, a, b, out, count, op, st); break;
    case BINE_C_DOUBLE_COMPLEX: e = batch_op<Cplx<double>>(n, a, b, out, count, op, st); break;
#endif
    default: return BINE_ERR_UNSUPPORTED;
  }
  if (e == hipErrorInvalidValue) return BINE_ERR_ARG;  // not co-aligned: caller falls back
  return e == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// system-coherent 16-B accesses of the direct transport (protocol notes at
// k_dm_move below); here because the tree body uses them too
// A 16-B store written through to memory (system coherent: sc0 sc1, and
// non-temporal) -- the stores into a peer's inbox slot.  Through a buffer
// resource (the compiler schedules it and tracks its counters; raw stride-0
// addressing, 2 GiB range, gfx9 untyped dword3 0x00020000) with the cache
// policy sc0 | sc1 | nt = 1 | 16 | 2; `base` is wave-uniform.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(void *base) {
  // the base is the same in every lane; readfirstlane says so to the compiler
  // (otherwise it wraps each store in a waterfall loop)
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint64_t u = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32 |
                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)u, (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, uint64_t vec, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(vec * 16), 0, 19);
}
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ----------------------------------------------------------------------------
// tree reduction: the owner's side of the flat reduce-scatter phase.  One
// launch evaluates the reference's whole reduction tree of a block from its P
// contributions (leaf 0 = the rank's own input, leaves 1..P-1 = the received
// blocks in tree order): HBM traffic (P + 1) * count * sizeof(T) instead of the
// 3 (P - 1) * count * sizeof(T) of P - 1 pairwise passes.  Per lane U 16-B
// vectors of every leaf in flight (NL * U loads), the tree evaluated in
// registers level by level -- v[i] = v[i] (op) v[i + w], left = inout -- so
// every element sees the reference's association and operand order.  Received
// leaves are read once: non-temporal loads.

struct TreeArgs {
  const void *leaf[kMaxLeaves];
  void *out;
  uint64_t head, nvec, n;
  int vec;        // 1: all operands co-aligned mod 16 B with `out`
  unsigned swap;  // bit l: level l combines v[i + w] (op) v[i] (the right side is inout)
};

// one level's combine; `sw` is wave-uniform (a scalar branch)
template <typename T, int OP>
__device__ __forceinline__ T comb(T l, T r, bool sw) { return sw ? apply<T, OP>(r, l) : apply<T, OP>(l, r); }
template <typename T, int OP>
__device__ __forceinline__ u32x4 comb16(u32x4 l, u32x4 r, bool sw) {
  return sw ? apply16<T, OP>(r, l) : apply16<T, OP>(l, r);
}

template <typename T, int OP, int NL>
__device__ __forceinline__ T tree_scalar(const TreeArgs &t, size_t i) {
  T v[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) v[j] = ((const T *)t.leaf[j])[i];
  int lvl = 0;
#pragma unroll
  for (int w = 1; w < NL; w <<= 1, lvl++)
#pragma unroll
    for (int j = 0; j < NL; j += 2 * w) v[j] = comb<T, OP>(v[j], v[j + w], (t.swap >> lvl) & 1);
  return v[0];
}

// Leaves are loaded and reduced in groups of G = min(NL, 8): positions
// [8g, 8g + 8) form a complete subtree of the reference's tree (levels w = 1,
// 2, 4), and the group results combine by the upper levels (w = 8) exactly
// as the leaves would.  U vectors of each leaf per lane in flight (tree_nl).  One tile of kBlock * U vectors per workgroup, no
// grid-stride loop, unguarded loads in every full tile (measured on MI355X,
// tools/tree_variants.hip: a grid-strided form with a guard on every load ran
// 31 us vs 24.5 us for 8 x 16 MiB).
template <typename T, int OP, int NL, int U, bool GUARD>
__device__ __forceinline__ void tree_tile(const u32x4 *const *lp, u32x4 *vo, size_t base, size_t nvec,
                                          unsigned swap) {
  constexpr int G = NL < 8 ? NL : 8, NG = NL / G, LG = G == 2 ? 1 : G == 4 ? 2 : 3;
  u32x4 part[U][NG];
#pragma unroll
  for (int g = 0; g < NG; g++) {
    u32x4 v[U][G];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * kBlock;
      if (!GUARD || i < nvec) {
        // tree position 0: plain load; positions 1..NL-1: non-temporal.  The
        // rank's own leaf sits at position `pos` of the primitive, which is 0
        // only on some ranks, so this is "one plain + NL-1 non-temporal
        // streams", not "own leaf cached": at the C3 chunk (16 MiB per leaf)
        // no leaf is L2-resident anyway, and the mix measured fastest
        // (tools/tree_variants.hip).  Two separate statements: a select
        // between the two loads of one address is folded into one plain load.
        if (g == 0) v[u][0] = lp[0][i];
#pragma unroll
        for (int j = g == 0 ? 1 : 0; j < G; j++) v[u][j] = __builtin_nontemporal_load(lp[g * G + j] + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      int lvl = 0;
#pragma unroll
      for (int w = 1; w < G; w <<= 1, lvl++)
#pragma unroll
        for (int j = 0; j < G; j += 2 * w) v[u][j] = comb16<T, OP>(v[u][j], v[u][j + w], (swap >> lvl) & 1);
      part[u][g] = v[u][0];
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    int lvl = LG;
#pragma unroll
    for (int w = 1; w < NG; w <<= 1, lvl++)
#pragma unroll
      for (int g = 0; g < NG; g += 2 * w) part[u][g] = comb16<T, OP>(part[u][g], part[u][g + w], (swap >> lvl) & 1);
    const size_t i = base + (size_t)u * kBlock;
    // non-temporal stores: 23.91 vs 24.12 us at the C3 chunk shape, 0.99 of
    // the 9 streams' read-only ceiling (profiles/r3_tree_variants.txt); nt
    // stores keep the line in the XCD's L2 for the allgather that sends it
    if (!GUARD || i < nvec) __builtin_nontemporal_store(part[u][0], vo + i);
  }
}

// elements before the 16-B aligned body and after its last vector (one
// workgroup; launched only when there are any: keeping this code out of the
// body kernel keeps its register count -- and occupancy -- at the body's own)
template <typename T, int OP, int NL>
__global__ __launch_bounds__(kBlock) void k_reduce_tree_edges(TreeArgs t) {
  constexpr size_t V = 16 / sizeof(T);
  T *out = (T *)t.out;
  for (size_t i = threadIdx.x; i < t.head; i += kBlock) out[i] = tree_scalar<T, OP, NL>(t, i);
  for (size_t i = t.head + t.nvec * V + threadIdx.x; i < t.n; i += kBlock) out[i] = tree_scalar<T, OP, NL>(t, i);
}

template <typename T, int OP, int NL, int U>
__global__ __launch_bounds__(kBlock) void k_reduce_tree(TreeArgs t) {
  T *out = (T *)t.out;
  // leaf base pointers into registers once (loading them from the kernel
  // arguments inside guarded loads put an s_waitcnt in front of every load)
  const u32x4 *lp[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) lp[j] = reinterpret_cast<const u32x4 *>((const T *)t.leaf[j] + t.head);
  u32x4 *vo = reinterpret_cast<u32x4 *>(out + t.head);
  const size_t base = (size_t)blockIdx.x * kBlock * U + threadIdx.x;
  if ((size_t)(blockIdx.x + 1) * kBlock * U <= t.nvec) tree_tile<T, OP, NL, U, false>(lp, vo, base, t.nvec, t.swap);
  else tree_tile<T, OP, NL, U, true>(lp, vo, base, t.nvec, t.swap);
}

// operands not co-aligned mod 16 B: scalar grid-stride
template <typename T, int OP, int NL>
__global__ __launch_bounds__(kBlock) void k_reduce_tree_scalar(TreeArgs t) {
  T *out = (T *)t.out;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < t.n; i += (size_t)gridDim.x * kBlock)
    out[i] = tree_scalar<T, OP, NL>(t, i);
}

template <typename T, int OP, int NL>
static hipError_t tree_nl(TreeArgs &t, hipStream_t st) {
  constexpr int U = NL == 2 ? 8 : NL <= 8 ? 4 : 2;  // tools/tree_variants.hip: <8,4> 25.2 us, <8,2> 26.5 us
  if (t.vec) {
    constexpr size_t V = 16 / sizeof(T);
    const size_t tiles = (t.nvec + (size_t)kBlock * U - 1) / ((size_t)kBlock * U);
    if (tiles) hipLaunchKernelGGL((k_reduce_tree<T, OP, NL, U>), dim3((unsigned)tiles), dim3(kBlock), 0, st, t);
    if (t.head || t.head + t.nvec * V < t.n)
      hipLaunchKernelGGL((k_reduce_tree_edges<T, OP, NL>), dim3(1), dim3(kBlock), 0, st, t);
  } else {
    size_t blocks = (t.n + kBlock * 4 - 1) / (kBlock * 4);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL((k_reduce_tree_scalar<T, OP, NL>), dim3((unsigned)blocks), dim3(kBlock), 0, st, t);
  }
  return hipGetLastError();
}

template <typename T, int OP>
static hipError_t tree_t(int nl, TreeArgs &t, hipStream_t st) {
  switch (nl) {
    case 2: return tree_nl<T, OP, 2>(t, st);
    case 4: return tree_nl<T, OP, 4>(t, st);
    case 8: return tree_nl<T, OP, 8>(t, st);
    case 16: return tree_nl<T, OP, 16>(t, st);
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
static hipError_t tree_op(int nl, TreeArgs &t, int op, hipStream_t st) {
  constexpr size_t V = 16 / sizeof(T);
  const uintptr_t oo = (uintptr_t)t.out;
  bool co = (oo % sizeof(T)) == 0;
  for (int j = 0; j < nl; j++) co = co && (((uintptr_t)t.leaf[j] ^ oo) & 15) == 0;
  t.vec = co ? 1 : 0;
  t.head = co ? std::min<uint64_t>(((16 - (oo & 15)) & 15) / sizeof(T), t.n) : t.n;
  t.nvec = co ? (t.n - t.head) / V : 0;
#define CALL(OP) tree_t<T, OP>(nl, t, st)
  BINE_OP_SWITCH(T, CALL)
#undef CALL
}

int BINE_FN(launch_reduce_tree)(int nl, const void *const *leaf, void *out, size_t count, int dtype, int op,
                                void *stream, unsigned swap) {
  if (count == 0) return BINE_SUCCESS;
#if BINE_OPSET == 0
  if (ext_op(dtype, op)) return launch_reduce_tree_logic(nl, leaf, out, count, dtype, op, stream, swap);
#endif
  if (nl < 2 || nl > kMaxLeaves || (nl & (nl - 1))) return BINE_ERR_ARG;
  size_t scale;
  dtype = canon_dtype(dtype, op, &scale);
  if (dtype < 0) return BINE_ERR_ARG;
  TreeArgs t{};
  for (int j = 0; j < nl; j++) t.leaf[j] = leaf[j];
  t.out = out;
  t.n = count * scale;
  t.swap = swap;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case BINE_INT8: e = tree_op<int8_t>(nl, t, op, st); break;
    case BINE_UINT8: e = tree_op<uint8_t>(nl, t, op, st); break;
    case BINE_INT16: e = tree_op<int16_t>(nl, t, op, st); break;
    case BINE_UINT16: e = tree_op<uint16_t>(nl, t, op, st); break;
    case BINE_INT32: e = tree_op<int32_t>(nl, t, op, st); break;
    case BINE_UINT32: e = tree_op<uint32_t>(nl, t, op, st); break;
    case BINE_INT64: e = tree_op<int64_t>(nl, t, op, st); break;
    case BINE_UINT64: e = tree_op<uint64_t>(nl, t, op, st); break;
    case BINE_FLOAT: e = tree_op<float>(nl, t, op, st); break;
    case BINE_DOUBLE: e = tree_op<double>(nl, t, op, st); break;
#if BINE_OPSET == 1
    case BINE_FLOAT_INT: e = tree_op<Pair<float>>(nl, t, op, st); break;
    case BINE_DOUBLE_INT: e = tree_op<Pair<double>>(nl, t, op, st); break;
    case BINE_LONG_INT: e = tree_op<Pair<long>>(nl, t, op, st); break;
    case BINE_2INT: e = tree_op<Pair<int>>(nl, t, op, st); break;
    case BINE_SHORT_INT: e = tree_op<Pair<short>>(nl, t, op, st); break;
    case BINE_C_FLOAT_COMPLEX: e = tree_op<Cplx<float>>(nl, t, op, st); break;
    case BINE_C_DOUBLE_COMPLEX: e = tree_op<Cplx<double>>(nl, t, op, st); break;
#endif
    default: return BINE_ERR_UNSUPPORTED;
  }
  return e == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

#if BINE_OPSET == 0
// ----------------------------------------------------------------------------
// direct peer-memory transport (bine_comm_set_direct, direct.cpp): one launch
// moves up to kMaxDm messages, `wgs` workgroups each.  A message's sequence
// number is seq = base[peer] + j + 1, base = this rank's count of earlier
// sub-messages to (push) or from (pull) that peer, kept in its own inbox and
// advanced by the launch's last workgroup; slot = seq mod kSlots.  Everything
// else follows from (seq, peer): the slot in the receiver's inbox, the flag to
// wait on -- push: the receiver's ack of the slot's previous use (seq -
// kSlots); pull: the sender's ready mark for seq -- and the flag to publish.
// Thread 0 of each workgroup polls the wait flag with a time limit; the
// workgroup copies its grid-strided share; every workgroup counts itself in;
// the last one of the message resets the counter for the slot's next use and
// publishes seq in the peer's inbox.  A wait that times out marks the
// transport poisoned; every later launch then exits at once, so no wait
// outlives the time limit.  No host-side state: launches can be captured and
// replayed.
//
// Memory protocol (round 4).  Bytes stored into a peer's inbox slot are
// written THROUGH to memory (global_store_dwordx4 ... sc0 sc1 nt: system
// coherent, so no L2 keeps them dirty); a workgroup waits for its stores'
// acknowledgements (vmcnt 0) before it counts itself in with a RELAXED
// system-scope atomic, and the last arriver publishes the flag with a relaxed
// system-scope store -- the flag is issued after every byte of the message
// was acknowledged.  No L2 write-back anywhere: round 3 released every
// workgroup's stores with buffer_wbl2 sc0 sc1, and those write-backs
// serialise -- a 16 MiB message by 512 workgroups took 47 us with them and
// 9.4 us written through (5.9 us with no protocol at all;
// profiles/r4_fence_probe.txt).  A reader polls with relaxed system-scope
// loads; once the flag is seen, its thread 0 invalidates once (the acquire
// fence: buffer_inv sc0 sc1, waited for) before the workgroup barrier -- the
// invalidation is of the CU's L1 and the XCD's L2, shared by every wave of
// the workgroup -- and the waves then read the slot with ordinary
// non-temporal loads.

__device__ __forceinline__ uint64_t ld_rlx_sys(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// thread 0 of a reader, after it saw the flag: one system-scope acquire
// (invalidation), completed before the workgroup barrier that follows
__device__ __forceinline__ void acquire_once() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  vm_wait();
}
// the end of a workgroup's share of a message: its stores acknowledged, then
// counted in (relaxed); true on the message's last arriver (thread 0 only)
__device__ __forceinline__ bool count_in(uint32_t *cnt, uint32_t nwg) {
  vm_wait();
  __syncthreads();
  if (threadIdx.x != 0) return false;
  const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (old + 1 != nwg) return false;
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the slot's next use: a later launch
  return true;
}
__device__ __forceinline__ void publish(uint64_t *flag, uint64_t seq) {
  __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// diagnostics (BINE_DIRECT_STAMPS, DmArgs::stamps): thread 0 of a workgroup
// appends its (entry, wait done, copy done) wall_clock64 stamps
__device__ __forceinline__ void dm_stamp(uint64_t *st, uint32_t serial, int kind, int msg, int wg, uint64_t t0,
                                         uint64_t t1, uint64_t t2) {
  if (!st) return;
  const uint64_t i = __hip_atomic_fetch_add(st, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (i >= st[1]) return;
  uint64_t *r = st + dm::kStampHdr + i * dm::kStampWords;
  r[0] = (uint64_t)serial << 32 | (uint64_t)kind << 24 | (uint64_t)(msg & 255) << 16 | (uint64_t)(wg & 0xffff);
  r[1] = t0;
  r[2] = t1;
  r[3] = t2;
}

// A wait that timed out: poison the transport -- the
// inbox word every later launch checks and the mapped host word the host
// reads -- and, for the first waiter of this rank to time out (the one whose
// exchange flips the inbox word), leave what it waited for in the host words
// (dm::TimeoutRecord, read by DirectState::describe): which kernel and phase,
// the peer, the slot, the sequence number wanted and the flag value last
// seen, the launch's serial, the workgroup and how long it waited.  Only
// that waiter sets the host word, after its record (release), so a host that
// sees the word set sees the record (a later waiter setting the word could
// let the host see it before the first one's record had landed).
__device__ __noinline__ void dm_time_out(uint32_t *poison, uint32_t *host, uint32_t kind, uint32_t phase, int rank,
                                         int peer, uint64_t slot, uint64_t want, uint64_t seen, uint32_t serial,
                                         uint64_t waited) {
  const uint32_t was = __hip_atomic_exchange(poison, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (!host) return;
  if (was == 0) {
    uint64_t *h = reinterpret_cast<uint64_t *>(host);
    const uint64_t v[dm::kRecWords] = {(uint64_t)kind << 8 | phase,
                                       (uint64_t)(uint32_t)rank,
                                       (uint64_t)(uint32_t)peer,
                                       slot,
                                       want,
                                       seen,
                                       serial,
                                       (uint64_t)blockIdx.x << 16 | threadIdx.x,
                                       waited};
#pragma unroll
    for (int i = 0; i < dm::kRecWords; i++)
      __hip_atomic_store(h + dm::kRecFirst + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one workgroup's share of message mi (workgroup wi of a.wgs): wait, copy,
// release, count in; the last workgroup of the message publishes.  false: the
// transport is poisoned (the workgroup must leave the launch at once)
__device__ __forceinline__ bool dm_copy_msg(const DmArgs &a, int mi, int wi, int nwg) {
  using namespace dm;
  const DmMsg &m = a.m[mi];
  uint8_t *own = a.own;
  uint32_t *poison = reinterpret_cast<uint32_t *>(own + kPoisonOff);
  uint64_t *base = reinterpret_cast<uint64_t *>(own + (m.push ? kBaseSendOff : kBaseRecvOff)) + m.peer;
  const uint64_t seq = __hip_atomic_load(base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)m.j + 1;
  const size_t k = (size_t)(seq % kSlots);
  uint8_t *remote = reinterpret_cast<uint8_t *const *>(own + kPeerTabOff)[m.peer];
  const size_t data_off = kFlagsBytes;
  const uint8_t *src;
  uint8_t *dst;
  const uint64_t *wait_ptr;
  uint64_t wait_val;
  uint64_t *sig_ptr;
  uint32_t *cnt_ptr;
  if (m.push) {
    src = m.src;
    dst = remote + data_off + ((size_t)a.rank * kSlots + k) * a.slot;
    wait_ptr = seq > (uint64_t)kSlots ? reinterpret_cast<const uint64_t *>(own + kAckOff + ((size_t)m.peer * kSlots + k) * kFlagStride)
                                      : nullptr;
    wait_val = seq - kSlots;
    sig_ptr = reinterpret_cast<uint64_t *>(remote + kReadyOff + ((size_t)a.rank * kSlots + k) * kFlagStride);
    cnt_ptr = reinterpret_cast<uint32_t *>(own + kCntPushOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
  } else {
    src = own + data_off + ((size_t)m.peer * kSlots + k) * a.slot;
    dst = m.dst;
    wait_ptr = reinterpret_cast<const uint64_t *>(own + kReadyOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
    wait_val = seq;
    sig_ptr = reinterpret_cast<uint64_t *>(remote + kAckOff + ((size_t)a.rank * kSlots + k) * kFlagStride);
    cnt_ptr = reinterpret_cast<uint32_t *>(own + kCntPullOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
  }
  __shared__ int go;
  uint64_t t0 = 0, t1 = 0;
  if (threadIdx.x == 0) {
    if (a.stamps) t0 = wall_clock64();
    int ok = __hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0;
    if (ok && wait_ptr) {
      const long long w0 = wall_clock64();
      uint64_t seen;
      while ((seen = ld_rlx_sys(wait_ptr)) < wait_val) {
        if (wall_clock64() - w0 > (long long)a.timeout_ticks) {
          dm_time_out(poison, a.poison_host, m.push ? dm::kWaitMovePush : dm::kWaitMovePull, 0, a.rank, m.peer, k,
                      wait_val, seen, a.serial, wall_clock64() - w0);
          ok = 0;
          break;
        }
        if (__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    // a pull reads what the peer wrote into our slot: one acquire; a push
    // only writes the slot the peer acknowledged (its reads were complete
    // before it counted in), nothing to acquire
    if (ok && !m.push) acquire_once();
    go = ok;
    if (a.stamps) t1 = wall_clock64();
  }
  __syncthreads();
  if (!go) return false;  // poisoned: the transport is dead, counters and bases no longer matter
  // grid-strided 16-B vectors (src / dst co-aligned mod 16: slots and plan
  // offsets are), bytes before the first boundary and after the last vector
  // by workgroup 0
  const size_t head = std::min<uint64_t>((16 - ((uintptr_t)dst & 15)) & 15, m.bytes);
  const size_t nvec = (m.bytes - head) / 16;
  if (wi == 0) {
    // a push's bytes into the slot written through too (system-scope byte
    // stores); a pull reads them after the acquire above
    auto put = [&](size_t i) {
      if (m.push) __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else dst[i] = src[i];
    };
    for (size_t i = threadIdx.x; i < head; i += kBlock) put(i);
    for (size_t i = head + nvec * 16 + threadIdx.x; i < m.bytes; i += kBlock) put(i);
  }
  const u32x4 *vs = reinterpret_cast<const u32x4 *>(src + head);
  u32x4 *vd = reinterpret_cast<u32x4 *>(dst + head);
  constexpr int U = 4;
  const size_t stride = (size_t)nwg * kBlock * U;
  if (m.push) {
    const __amdgpu_buffer_rsrc_t r = wt_rsrc(vd);  // (a push's head is empty: vd is the slot)
    for (size_t b0 = (size_t)wi * kBlock * U + threadIdx.x; b0 < nvec; b0 += stride) {
      u32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const size_t i = b0 + (size_t)u * kBlock;
        if (i < nvec) x[u] = __builtin_nontemporal_load(vs + i);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const size_t i = b0 + (size_t)u * kBlock;
        if (i < nvec) st_wt(r, i, x[u]);
      }
    }
  } else {
    for (size_t b0 = (size_t)wi * kBlock * U + threadIdx.x; b0 < nvec; b0 += stride) {
      u32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const size_t i = b0 + (size_t)u * kBlock;
        if (i < nvec) x[u] = __builtin_nontemporal_load(vs + i);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const size_t i = b0 + (size_t)u * kBlock;
        if (i < nvec) __builtin_nontemporal_store(x[u], vd + i);
      }
    }
  }
  // stores acknowledged (written through) / slot reads complete, count in; the
  // last one of the message publishes
  const bool last = count_in(cnt_ptr, (uint32_t)nwg);
  if (threadIdx.x == 0 && a.stamps) dm_stamp(a.stamps, a.serial, m.push ? 0 : 1, mi, wi, t0, t1, wall_clock64());
  if (last) publish(sig_ptr, seq);
  return true;
}

// one workgroup's share of a push GROUP led by message mi (the same bytes to
// several peers, DmMsg::grp): each member's slot-reuse acknowledgement is
// awaited, the source is read once and stored into every member's slot, and
// every member is counted in and published exactly as a standalone push
__device__ __forceinline__ bool dm_mcast_msg(const DmArgs &a, int mi, int wi, int nwg) {
  using namespace dm;
  uint8_t *own = a.own;
  uint32_t *poison = reinterpret_cast<uint32_t *>(own + kPoisonOff);
  __shared__ u32x4 *dv[kMaxDm];
  __shared__ uint64_t dseq[kMaxDm];
  __shared__ int dmem[kMaxDm];
  __shared__ int nd, go;
  if (threadIdx.x == 0) {
    int ok = __hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0;
    int n = 0;
    for (int j = 0; j < a.nmsg; j++) {
      const DmMsg &m = a.m[j];
      if (!m.push || m.grp != mi) continue;
      const uint64_t seq = __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + kBaseSendOff) + m.peer,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)m.j + 1;
      const size_t k = (size_t)(seq % kSlots);
      uint8_t *remote = reinterpret_cast<uint8_t *const *>(own + kPeerTabOff)[m.peer];
      dv[n] = reinterpret_cast<u32x4 *>(remote + kFlagsBytes + ((size_t)a.rank * kSlots + k) * a.slot);
      dseq[n] = seq;
      dmem[n] = j;
      n++;
      if (ok && seq > (uint64_t)kSlots) {
        const uint64_t *w = reinterpret_cast<const uint64_t *>(own + kAckOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
        const long long t0 = wall_clock64();
        uint64_t seen;
        while ((seen = ld_rlx_sys(w)) < seq - kSlots) {
          if (wall_clock64() - t0 > (long long)a.timeout_ticks) {
            dm_time_out(poison, a.poison_host, dm::kWaitGroupPush, 0, a.rank, m.peer, k, seq - kSlots, seen, a.serial,
                        wall_clock64() - t0);
            ok = 0;
            break;
          }
          if (__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    nd = n;
    go = ok;
  }
  __syncthreads();
  if (!go) return false;  // (writes only into acknowledged slots: nothing to acquire)
  const DmMsg &L = a.m[mi];
  const uint8_t *src = L.src;
  const int n = nd;
  // every slot is 16-B aligned (a multiple of 4 KiB from the inbox base):
  // whole vectors from byte 0, the tail bytes by workgroup 0
  const size_t nvec = L.bytes / 16;
  if (wi == 0)
    for (int d = 0; d < n; d++)
      for (size_t i = nvec * 16 + threadIdx.x; i < L.bytes; i += kBlock)
        __hip_atomic_store(reinterpret_cast<uint8_t *>(dv[d]) + i, src[i], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  const u32x4 *vs = reinterpret_cast<const u32x4 *>(src);
  constexpr int U = 4;
  const size_t stride = (size_t)nwg * kBlock * U;
  for (size_t b0 = (size_t)wi * kBlock * U + threadIdx.x; b0 < nvec; b0 += stride) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = b0 + (size_t)u * kBlock;
      if (i < nvec) x[u] = __builtin_nontemporal_load(vs + i);
    }
    for (int d = 0; d < n; d++) {
      const __amdgpu_buffer_rsrc_t r = wt_rsrc(dv[d]);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const size_t i = b0 + (size_t)u * kBlock;
        if (i < nvec) st_wt(r, i, x[u]);
      }
    }
  }
  vm_wait();  // every member's bytes acknowledged (written through)
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int d = 0; d < n; d++) {
      const DmMsg &m = a.m[dmem[d]];
      const size_t k = (size_t)(dseq[d] % kSlots);
      uint32_t *cnt = reinterpret_cast<uint32_t *>(own + kCntPushOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
      const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old + 1 == (uint32_t)nwg) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint8_t *remote = reinterpret_cast<uint8_t *const *>(own + kPeerTabOff)[m.peer];
        publish(reinterpret_cast<uint64_t *>(remote + kReadyOff + ((size_t)a.rank * kSlots + k) * kFlagStride),
                dseq[d]);
      }
    }
  }
  return true;
}

// copy workgroup b of the launch: the entry of DmArgs::cidx it belongs to
// (entry c has cwgs[c] workgroups: wgs for a message alone, wgs x members for
// a push group, so a group keeps the parallelism of its members), then its
// message alone or the group it leads
__device__ __forceinline__ bool dm_copy_wg(const DmArgs &a, unsigned b) {
  int c = 0;
  unsigned start = 0;
  while (c + 1 < a.ncopy && b >= start + (unsigned)a.cwgs[c]) start += (unsigned)a.cwgs[c++];
  const int mi = a.cidx[c], wi = (int)(b - start), nwg = a.cwgs[c];
  return a.m[mi].push && a.m[mi].grp == mi ? dm_mcast_msg(a, mi, wi, nwg) : dm_copy_msg(a, mi, wi, nwg);
}

// thread 0, after its workgroup's share of the launch: the last workgroup of
// the launch advances the sequence bases of every message (every workgroup has
// read them; the next launch is stream-ordered after this one)
__device__ __forceinline__ void dm_launch_done(const DmArgs &a) {
  using namespace dm;
  if (threadIdx.x != 0) return;
  uint8_t *own = a.own;
  uint32_t *lc = reinterpret_cast<uint32_t *>(own + kLaunchCntOff);
  // relaxed: every workgroup read its bases before it got here (the values
  // fed its addresses), and the next launch follows in stream order
  const uint32_t ol = __hip_atomic_fetch_add(lc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ol + 1 == gridDim.x) {
    __hip_atomic_store(lc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; i < a.nmsg; i++) {
      uint64_t *bp = reinterpret_cast<uint64_t *>(own + (a.m[i].push ? kBaseSendOff : kBaseRecvOff)) + a.m[i].peer;
      __hip_atomic_store(bp, __hip_atomic_load(bp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_dm_move(DmArgs a) {
  if (!dm_copy_wg(a, blockIdx.x)) return;
  dm_launch_done(a);
}

// every message: in range; copied by its own workgroups (cidx, each once),
// carried by its group's leader (a push with the leader's bytes and source),
// or -- tree launches -- a leaf; false otherwise
static bool dm_args_ok(const DmArgs &a, bool leaves_ok) {
  if (a.nmsg <= 0 || a.nmsg > kMaxDm || a.wgs < 1 || !a.own || !a.slot || a.ncopy < 0 || a.ncopy > a.nmsg)
    return false;
  uint64_t seen = 0;
  int ncw = 0;
  for (int c = 0; c < a.ncopy; c++) {
    const int i = a.cidx[c];
    if (i < 0 || i >= a.nmsg || (seen >> i & 1) || a.m[i].leaf >= 0 || (a.m[i].grp >= 0 && a.m[i].grp != i) ||
        a.cwgs[c] < 1 || a.cwgs[c] > 1 << 16)
      return false;
    seen |= 1ull << i;
    ncw += a.cwgs[c];
  }
  if (ncw != a.ncw) return false;
  for (int i = 0; i < a.nmsg; i++) {
    const DmMsg &m = a.m[i];
    if (m.peer < 0 || m.peer >= dm::kMaxPeers || m.j < 0 || m.j >= dm::kSlots || m.bytes > a.slot) return false;
    if (m.grp >= 0) {
      if (!m.push || m.grp >= a.nmsg || !(seen >> m.grp & 1) || a.m[m.grp].grp != m.grp ||
          a.m[m.grp].src != m.src || a.m[m.grp].bytes != m.bytes)
        return false;
    } else if (!(seen >> i & 1) && !(leaves_ok && m.leaf >= 0)) {
      return false;
    }
  }
  return true;
}

// blocks per CU a direct-transport launch leaves free (dm_residency_cap)
static int dm_margin() {
  static const int m = [] {
    const char *e = getenv("BINE_DIRECT_RESIDENCY_MARGIN");
    return e && *e ? std::max(0, atoi(e)) : 1;
  }();
  return m;
}

// Workgroup slots one direct-transport launch may take on the current device
// (bine_internal.h dm_fit_residency, dm_residency_cap): CUs x (resident blocks
// per CU of kernel `k` (the occupancy API: registers, LDS, wave slots) -
// margin) / share; 0 if unknown.  Both factors are queried once per kernel
// and device.
static int dm_cap(const void *k, int share) {
  static std::mutex mu;
  static std::map<std::pair<const void *, int>, std::pair<int, int>> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find({k, dev});
  if (it == cache.end()) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, kBlock, 0) != hipSuccess) {
      (void)hipGetLastError();
      cus = per = 0;
    }
    it = cache.emplace(std::make_pair(k, dev), std::make_pair(cus, per)).first;
  }
  return dm_residency_cap(it->second.first, it->second.second, dm_margin(), share);
}

int launch_dm_move(const DmArgs &a0, void *stream) {
  if (a0.nmsg <= 0) return BINE_SUCCESS;
  if (!dm_args_ok(a0, false)) return BINE_ERR_ARG;
  DmArgs a = a0;
  if (dm_fit_residency(a.cwgs, a.ncopy, nullptr, dm_cap((const void *)k_dm_move, a.share)) > 0) {
    a.ncw = 0;
    for (int c = 0; c < a.ncopy; c++) a.ncw += a.cwgs[c];
  }
  hipLaunchKernelGGL(k_dm_move, dim3((unsigned)a.ncw), dim3(kBlock), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// k_dm_move_tree<T, OP, NL> (bine_internal.h DmTree): the copy messages as in
// k_dm_move, then `twgs` workgroups that evaluate the flat reduce-scatter's
// tree straight out of the leaf pulls' inbox slots
template <typename T, int OP, int NL>
__global__ __launch_bounds__(kBlock) void k_dm_move_tree(DmArgs a, DmTree t) {
  using namespace dm;
  const unsigned ncw = (unsigned)a.ncw;
  if (blockIdx.x < ncw) {
    if (!dm_copy_wg(a, blockIdx.x)) return;
    dm_launch_done(a);
    return;
  }
  uint8_t *own = a.own;
  uint32_t *poison = reinterpret_cast<uint32_t *>(own + kPoisonOff);
  // every leaf: its slot in our inbox, the sender's ready mark to wait for
  // -- polled side by side, lane j for leaf j in one loop (one flag round
  // trip, not one per leaf)
  const u32x4 *lp[NL];
  const uint64_t *wp = nullptr;
  uint64_t wseq = 0;
  int wpeer = -1;
  size_t wslot = 0;
  __shared__ int go;
  uint64_t t0 = 0, t1 = 0;
  if (threadIdx.x == 0) {
    if (a.stamps) t0 = wall_clock64();
    go = __hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NL; j++) {
    if (j == t.pos) {
      lp[j] = reinterpret_cast<const u32x4 *>(t.own_leaf);
      continue;
    }
    const DmMsg &m = a.m[t.leaf_msg[j]];
    const uint64_t seq = __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + kBaseRecvOff) + m.peer,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)m.j + 1;
    const size_t k = (size_t)(seq % kSlots);
    lp[j] = reinterpret_cast<const u32x4 *>(own + kFlagsBytes + ((size_t)m.peer * kSlots + k) * a.slot);
    if ((int)threadIdx.x == j) {
      wp = reinterpret_cast<const uint64_t *>(own + kReadyOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
      wseq = seq;
      wpeer = m.peer;
      wslot = k;
    }
  }
  if (wp && go) {
    const long long tw = wall_clock64();
    uint64_t seen;
    while ((seen = ld_rlx_sys(wp)) < wseq) {
      if (wall_clock64() - tw > (long long)a.timeout_ticks) {
        dm_time_out(poison, a.poison_host, dm::kWaitTreeLeaf, 0, a.rank, wpeer, wslot, wseq, seen, a.serial,
                    wall_clock64() - tw);
        go = 0;
        break;
      }
      if (__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        go = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();  // every leaf's poll has completed
  if (threadIdx.x == 0) {
    if (go) acquire_once();  // every leaf's mark seen: what the senders wrote before it
    if (a.stamps) t1 = wall_clock64();
  }
  __syncthreads();
  if (!go) return;
  // the tree over this workgroup's tiles (k_reduce_tree's tile body).  Fewer
  // vectors in flight per lane than k_reduce_tree: the copy workgroups of the
  // launch get this kernel's register allocation too
  constexpr int U = NL <= 4 ? 4 : NL == 8 ? 2 : 1;
  const int tw = (int)(blockIdx.x - ncw);
  u32x4 *vo = reinterpret_cast<u32x4 *>(t.out);
  const size_t tile = (size_t)kBlock * U, ntiles = (t.nvec + tile - 1) / tile;
  for (size_t ti = (size_t)tw; ti < ntiles; ti += (size_t)t.twgs) {
    const size_t b = ti * tile + threadIdx.x;
    if ((ti + 1) * tile <= t.nvec) tree_tile<T, OP, NL, U, false>(lp, vo, b, t.nvec, t.swap);
    else tree_tile<T, OP, NL, U, true>(lp, vo, b, t.nvec, t.swap);
  }
  // every leaf slice read (loads complete): count in per leaf; the last tree
  // workgroup of a leaf acknowledges its slot to the sender (as a pull's last
  // workgroup does)
  vm_wait();
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.stamps) dm_stamp(a.stamps, a.serial, 2, 255, tw, t0, t1, wall_clock64());
#pragma unroll
    for (int j = 0; j < NL; j++) {
      if (j == t.pos) continue;
      const DmMsg &m = a.m[t.leaf_msg[j]];
      const uint64_t seq = __hip_atomic_load(reinterpret_cast<const uint64_t *>(own + kBaseRecvOff) + m.peer,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)m.j + 1;
      const size_t k = (size_t)(seq % kSlots);
      uint32_t *cnt = reinterpret_cast<uint32_t *>(own + kCntPullOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
      const uint32_t old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (old + 1 == (uint32_t)t.twgs) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint8_t *remote = reinterpret_cast<uint8_t *const *>(own + kPeerTabOff)[m.peer];
        publish(reinterpret_cast<uint64_t *>(remote + kAckOff + ((size_t)a.rank * kSlots + k) * kFlagStride), seq);
      }
    }
  }
  dm_launch_done(a);
}

bool dm_tree_supported(int dtype, int op, int nl) {
  return dm_fused_supported(dtype, op) && (nl == 2 || nl == 4 || nl == 8 || nl == 16);
}

template <typename T, int OP>
static const void *dmt_kernel(int nl) {
  switch (nl) {
    case 2: return (const void *)k_dm_move_tree<T, OP, 2>;
    case 4: return (const void *)k_dm_move_tree<T, OP, 4>;
    case 8: return (const void *)k_dm_move_tree<T, OP, 8>;
    case 16: return (const void *)k_dm_move_tree<T, OP, 16>;
    default: return nullptr;
  }
}

template <typename T, int OP>
static hipError_t dmt_launch(const DmArgs &a0, const DmTree &t0, hipStream_t st) {
  DmArgs a = a0;
  DmTree t = t0;
  if (const void *k = dmt_kernel<T, OP>(t.nl))
    if (dm_fit_residency(a.cwgs, a.ncopy, &t.twgs, dm_cap(k, a.share)) > 0) {
      a.ncw = 0;
      for (int c = 0; c < a.ncopy; c++) a.ncw += a.cwgs[c];
    }
  const dim3 g((unsigned)(a.ncw + t.twgs));
  switch (t.nl) {
    case 2: hipLaunchKernelGGL((k_dm_move_tree<T, OP, 2>), g, dim3(kBlock), 0, st, a, t); break;
    case 4: hipLaunchKernelGGL((k_dm_move_tree<T, OP, 4>), g, dim3(kBlock), 0, st, a, t); break;
    case 8: hipLaunchKernelGGL((k_dm_move_tree<T, OP, 8>), g, dim3(kBlock), 0, st, a, t); break;
    case 16: hipLaunchKernelGGL((k_dm_move_tree<T, OP, 16>), g, dim3(kBlock), 0, st, a, t); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
static hipError_t dmt_t(const DmArgs &a, const DmTree &t, int op, hipStream_t st) {
#define CALL(OP) dmt_launch<T, OP>(a, t, st)
  BINE_OP_SWITCH(T, CALL)
#undef CALL
}

int launch_dm_move_tree(const DmArgs &a, const DmTree &t, int dtype, int op, void *stream) {
  if (!dm_tree_supported(dtype, op, t.nl)) return BINE_ERR_UNSUPPORTED;
  if (!dm_args_ok(a, true) || t.twgs < 1 || t.pos < 0 || t.pos >= t.nl || !t.nvec || t.nvec * 16 > a.slot ||
      !t.out || !t.own_leaf || ((uintptr_t)t.out & 15) || ((uintptr_t)t.own_leaf & 15))
    return BINE_ERR_ARG;
  // every leaf position but pos once, by a leaf pull of nvec vectors; no other leaves
  uint64_t seen = 0;
  int nleaf = 0;
  for (int i = 0; i < a.nmsg; i++) nleaf += a.m[i].leaf >= 0;
  if (nleaf != t.nl - 1) return BINE_ERR_ARG;
  for (int j = 0; j < t.nl; j++) {
    if (j == t.pos) continue;
    const int i = t.leaf_msg[j];
    if (i < 0 || i >= a.nmsg || (seen >> i & 1) || a.m[i].push || a.m[i].leaf != j || a.m[i].bytes != t.nvec * 16)
      return BINE_ERR_ARG;
    seen |= 1ull << i;
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case BINE_FLOAT: e = dmt_t<float>(a, t, op, st); break;
    case BINE_DOUBLE: e = dmt_t<double>(a, t, op, st); break;
    case BINE_INT32: e = dmt_t<int32_t>(a, t, op, st); break;
    case BINE_INT64: e = dmt_t<int64_t>(a, t, op, st); break;
    case BINE_UINT32: e = dmt_t<uint32_t>(a, t, op, st); break;
    case BINE_UINT64: e = dmt_t<uint64_t>(a, t, op, st); break;
    default: return BINE_ERR_UNSUPPORTED;
  }
  return e == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// ----------------------------------------------------------------------------
// k_dm_fused: a flat-form small collective in one launch (bine_internal.h
// DmFusedArgs).  Flags, counters, slots and sequence bases are k_dm_move's.

namespace dmf {
using namespace dm;

// where message m of this launch reads, writes, waits and publishes
struct Msg {
  const u32x4 *src;
  u32x4 *dst;
  const uint64_t *wait;  // nullptr: nothing to wait for
  uint64_t wait_val;
  uint64_t *sig;
  uint32_t *cnt;
  uint64_t seq, nvec;
  // this workgroup's slice flags (bine_internal.h dm::kSliceReadyOff; null
  // when the launch has more workgroups than the layout holds): the one it
  // may wait on instead of `wait`, the one it sets after its slice, and (a
  // push) this rank's record of the slot's previous use
  const uint64_t *swait;
  uint64_t *ssig;
  uint64_t *geom;
  int k;
};

// a slice flag's value: the sequence number and the setter's workgroup count
__device__ __forceinline__ uint64_t slice_val(uint64_t seq, int wgs) {
  return seq << kSliceWgsBits | (uint64_t)wgs;
}

__device__ __forceinline__ Msg resolve(const DmFusedArgs &a, const DmMsg &m) {
  Msg r;
  uint8_t *own = a.own;
  const uint64_t *base = reinterpret_cast<const uint64_t *>(own + (m.push ? kBaseSendOff : kBaseRecvOff)) + m.peer;
  r.seq = __hip_atomic_load(base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)m.j + 1;
  const size_t k = (size_t)(r.seq % kSlots);
  r.k = (int)k;
  uint8_t *remote = reinterpret_cast<uint8_t *const *>(own + kPeerTabOff)[m.peer];
  r.nvec = m.bytes / 16;
  const bool sl = a.slices && a.wgs <= kSliceMax;
  const size_t w = blockIdx.x;
  if (m.push) {
    r.src = reinterpret_cast<const u32x4 *>(m.src);
    r.dst = reinterpret_cast<u32x4 *>(remote + kFlagsBytes + ((size_t)a.rank * kSlots + k) * a.slot);
    r.wait = r.seq > (uint64_t)kSlots
                 ? reinterpret_cast<const uint64_t *>(own + kAckOff + ((size_t)m.peer * kSlots + k) * kFlagStride)
                 : nullptr;
    r.wait_val = r.seq - kSlots;
    r.sig = reinterpret_cast<uint64_t *>(remote + kReadyOff + ((size_t)a.rank * kSlots + k) * kFlagStride);
    r.cnt = reinterpret_cast<uint32_t *>(own + kCntPushOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
    r.swait = sl ? reinterpret_cast<const uint64_t *>(own + kSliceAckOff + slice_off(w, (size_t)m.peer, k))
                 : nullptr;
    r.ssig = sl ? reinterpret_cast<uint64_t *>(remote + kSliceReadyOff + slice_off(w, (size_t)a.rank, k)) : nullptr;
    r.geom = reinterpret_cast<uint64_t *>(own + kGeomOff + ((size_t)m.peer * kSlots + k) * 16);
  } else {
    r.src = reinterpret_cast<const u32x4 *>(own + kFlagsBytes + ((size_t)m.peer * kSlots + k) * a.slot);
    r.dst = reinterpret_cast<u32x4 *>(m.dst);
    r.wait = reinterpret_cast<const uint64_t *>(own + kReadyOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
    r.wait_val = r.seq;
    r.sig = reinterpret_cast<uint64_t *>(remote + kAckOff + ((size_t)a.rank * kSlots + k) * kFlagStride);
    r.cnt = reinterpret_cast<uint32_t *>(own + kCntPullOff + ((size_t)m.peer * kSlots + k) * kFlagStride);
    r.swait = sl ? reinterpret_cast<const uint64_t *>(own + kSliceReadyOff + slice_off(w, (size_t)m.peer, k))
                 : nullptr;
    r.ssig = sl ? reinterpret_cast<uint64_t *>(remote + kSliceAckOff + slice_off(w, (size_t)a.rank, k)) : nullptr;
    r.geom = nullptr;
  }
  return r;
}

// whether this workgroup may go on with message m: the whole message's flag,
// or -- when both ends cut it with this launch's workgroup count -- the flag
// of its own slice.  A push's slice of the slot's previous use was acked by
// the receiver's workgroup w only for the bytes THAT message's cut gave it:
// usable when this rank's record says that use was a k_dm_fused push of the
// same vector count (same wgs: in the ack's value).  `seen` = the whole
// flag's last value (the time-out record's).
__device__ __forceinline__ bool flag_ok(const DmFusedArgs &a, const Msg &m, bool push, bool geom_ok, uint64_t *seen) {
  *seen = ld_rlx_sys(m.wait);
  if (*seen >= m.wait_val) return true;
  if (!m.swait || (push && !geom_ok)) return false;
  const uint64_t v = ld_rlx_sys(m.swait);
  return (v >> kSliceWgsBits) >= m.wait_val && (v & ((1u << kSliceWgsBits) - 1)) == (uint64_t)a.wgs;
}

// The waits and arrivals of a phase's messages run side by side, one thread
// per message: one flag round trip per phase instead of one per message
// (a small collective is a chain of such round trips).
//
// wait_all: thread t < n polls message first + t's flag (relaxed
// system-scope loads, bounded); after the barrier, when any of them is a
// ready mark (acq: its slot is read next), thread 0 acquires once -- every
// poll has completed before the barrier -- and a second barrier orders the
// workgroup's reads after it.  false: the transport is poisoned (now or
// earlier).
__device__ __forceinline__ bool wait_all(const DmFusedArgs &a, int first, int n, bool acq, uint32_t phase) {
  __shared__ int bad;
  uint32_t *poison = reinterpret_cast<uint32_t *>(a.own + kPoisonOff);
  if (threadIdx.x == 0) bad = __hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  __syncthreads();
  if ((int)threadIdx.x < n && !bad) {
    const DmMsg &mm = a.m[first + threadIdx.x];
    const Msg m = resolve(a, mm);
    if (m.wait) {
      const long long t0 = wall_clock64();
      uint64_t seen;
      // a push's slice acks cover this push's slice only if the slot's
      // previous use was a k_dm_fused push of the same vector count
      const bool geom_ok = mm.push && m.swait && ld_rlx_sys(m.geom) == m.wait_val &&
                           ld_rlx_sys(m.geom + 1) == m.nvec;
      while (!flag_ok(a, m, mm.push, geom_ok, &seen)) {
        if (wall_clock64() - t0 > (long long)a.timeout_ticks) {
          dm_time_out(poison, a.poison_host, mm.push ? dm::kWaitFusedPush : dm::kWaitFusedPull, phase, a.rank,
                      mm.peer, m.seq % kSlots, m.wait_val, seen, a.serial, wall_clock64() - t0);
          bad = 1;
          break;
        }
        if (__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          bad = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
  const bool ok = !bad;
  if (threadIdx.x == 0 && ok && acq && n) acquire_once();
  __syncthreads();  // the reads after the acquire; `bad` is reused by the next wait
  return ok;
}

// arrive_all: the workgroup's shares of messages first .. first + n - 1 are
// done (stores acknowledged, reads complete); thread t counts in for message
// t, and the last workgroup of a message publishes its seq (k_dm_move's
// protocol)
__device__ __forceinline__ void arrive_all(const DmFusedArgs &a, int first, int n) {
  vm_wait();
  __syncthreads();
  if ((int)threadIdx.x < n) {
    const DmMsg &mm = a.m[first + threadIdx.x];
    const Msg m = resolve(a, mm);
    // this workgroup's slice is done: its flag (the peer's workgroup w may go on)
    if (m.ssig) publish(m.ssig, slice_val(m.seq, a.wgs));
    const uint32_t old = __hip_atomic_fetch_add(m.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (old + 1 == (uint32_t)a.wgs) {
      __hip_atomic_store(m.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the slot's next use
      if (mm.push) {  // the use this push made of the slot (read by the slot's next push, a later launch)
        __hip_atomic_store(m.geom, m.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(m.geom + 1, m.nvec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      publish(m.sig, m.seq);
    }
  }
  __syncthreads();  // every thread's resolve() before thread 0's launch-counter add (the kernel's end)
}

// this workgroup's slice of a message of n vectors
__device__ __forceinline__ void slice(uint64_t n, int wgs, uint64_t *lo, uint64_t *hi) {
  *lo = n * blockIdx.x / (uint64_t)wgs;
  *hi = n * (blockIdx.x + 1) / (uint64_t)wgs;
}

// a push writes the peer's slot through; a pull reads its own slot after
// the acquire of wait_all.  U vectors per lane in flight (all loads, then
// all stores): with one, every store waits for its own load and the slice
// streams at a fraction of HBM bandwidth.
__device__ __forceinline__ void copy_slice(const Msg &m, int wgs, bool push) {
  constexpr int U = 4;
  uint64_t lo, hi;
  slice(m.nvec, wgs, &lo, &hi);
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(push ? m.dst : nullptr);
  for (uint64_t b = lo + threadIdx.x; b < hi; b += (uint64_t)kBlock * U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = b + (uint64_t)u * kBlock;
      if (i < hi) x[u] = __builtin_nontemporal_load(m.src + i);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = b + (uint64_t)u * kBlock;
      if (i < hi) {
        if (push) st_wt(r, i, x[u]);
        else __builtin_nontemporal_store(x[u], m.dst + i);
      }
    }
  }
}

// this workgroup's slice [lo, hi) of a tree of NL leaves (own leaf at `pos`:
// plain loads; the received ones in the inbox slots: non-temporal), each
// result vector stored to `out` and pushed from registers into the nc
// allgather slots; U vectors of every leaf per lane in flight, U x NL <= 8
// (the registers of the kernel's other phases)
template <typename T, int OP, int NL>
__device__ __forceinline__ void tree_slice(const u32x4 *const *lp, int nl, int pos, unsigned swap, u32x4 *out,
                                           const __amdgpu_buffer_rsrc_t *cp, int nc, uint64_t lo, uint64_t hi) {
  constexpr int U = NL >= 8 ? 1 : 8 / NL;
  for (uint64_t b = lo + threadIdx.x; b < hi; b += (uint64_t)kBlock * U) {
    u32x4 v[U][NL];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = b + (uint64_t)u * kBlock;
      if (i < hi) {
#pragma unroll
        for (int j = 0; j < NL; j++) {
          if (j >= nl) continue;  // a tree of nl <= NL leaves (a non-power-of-two P's)
          if (j == pos) v[u][j] = lp[j][i];
          else v[u][j] = __builtin_nontemporal_load(lp[j] + i);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = b + (uint64_t)u * kBlock;
      if (i >= hi) continue;
      int lvl = 0;
#pragma unroll
      for (int w = 1; w < NL; w <<= 1, lvl++)
#pragma unroll
        for (int j = 0; j < NL; j += 2 * w)
          if (j + w < nl) v[u][j] = comb16<T, OP>(v[u][j], v[u][j + w], (swap >> lvl) & 1);
      out[i] = v[u][0];
#pragma unroll
      for (int c = 0; c < kMaxFusedPeers; c++)
        if (c < nc) st_wt(cp[c], i, v[u][0]);
    }
  }
}
}  // namespace dmf

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void k_dm_fused(DmFusedArgs a) {
  using namespace dmf;
  const int nm = a.d0 + a.nd;
  const uint64_t t0 = a.stamps ? wall_clock64() : 0;
  // phase A: our blocks of every chunk into the peers' inboxes (each slot's
  // previous use acknowledged first)
  if (!wait_all(a, 0, a.na, false, 0)) return;
  const uint64_t t1 = a.stamps ? wall_clock64() : 0;
  // workgroup w starts at message w mod na and rotates: at any moment the
  // workgroups spread over every peer's link instead of all pushing to the
  // same peer first (on a node each peer is its own xGMI link)
  for (int k = 0; k < a.na; k++) {
    const int i = (int)((blockIdx.x + (unsigned)k) % (unsigned)a.na);
    copy_slice(resolve(a, a.m[i]), a.wgs, true);
  }
  arrive_all(a, 0, a.na);
  // phases B_c: the peers' blocks of chunk c, read in place in our inbox as
  // the tree's leaves; each result vector goes to `out` and, for the flat
  // allgather, straight from registers into every peer's slot -- whose
  // previous use must have been acknowledged first
  for (int ti = 0; ti < a.nt; ti++) {
    const DmFusedTree &t = a.t[ti];
    if (!wait_all(a, t.b0, t.nb + t.nc, t.nb > 0, 1 + ti)) return;
    const u32x4 *lp[kMaxLeaves];
#pragma unroll
    for (int j = 0; j < kMaxLeaves; j++)
      lp[j] = j >= a.nl ? nullptr
              : j == a.pos ? reinterpret_cast<const u32x4 *>(t.own_leaf)
                           : resolve(a, a.m[t.leaf[j]]).src;
    __amdgpu_buffer_rsrc_t cp[kMaxFusedPeers];
#pragma unroll
    for (int i = 0; i < kMaxFusedPeers; i++)
      if (i < t.nc) cp[i] = wt_rsrc(resolve(a, a.m[t.b0 + t.nb + i]).dst);
    u32x4 *out = reinterpret_cast<u32x4 *>(t.out);
    uint64_t lo, hi;
    slice(t.nvec, a.wgs, &lo, &hi);
    if (a.nl <= 2) tree_slice<T, OP, 2>(lp, a.nl, a.pos, a.swap, out, cp, t.nc, lo, hi);
    else if (a.nl <= 4) tree_slice<T, OP, 4>(lp, a.nl, a.pos, a.swap, out, cp, t.nc, lo, hi);
    else if (a.nl <= 8) tree_slice<T, OP, 8>(lp, a.nl, a.pos, a.swap, out, cp, t.nc, lo, hi);
    else tree_slice<T, OP, 16>(lp, a.nl, a.pos, a.swap, out, cp, t.nc, lo, hi);
    // every leaf slice is read (the senders may reuse their slots) and every
    // result slice is in the peers' inboxes
    arrive_all(a, t.b0, t.nb + t.nc);
  }
  // phase D: the peers' results out of our inbox
  if (!wait_all(a, a.d0, a.nd, true, 15)) return;
  for (int k = 0; k < a.nd; k++) {  // rotated as phase A (the slots lie in different HBM channels anyway)
    const int i = (int)((blockIdx.x + (unsigned)k) % (unsigned)a.nd);
    copy_slice(resolve(a, a.m[a.d0 + i]), a.wgs, false);
  }
  arrive_all(a, a.d0, a.nd);
  if (threadIdx.x == 0 && a.stamps) dm_stamp(a.stamps, a.serial, 4, 255, blockIdx.x, t0, t1, wall_clock64());
  // the launch's last workgroup advances the sequence bases (every workgroup
  // has read them: each resolve() happened before its launch-counter add)
  if (threadIdx.x == 0) {
    uint32_t *lc = reinterpret_cast<uint32_t *>(a.own + dm::kLaunchCntOff);
    const uint32_t ol = __hip_atomic_fetch_add(lc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ol + 1 == gridDim.x) {
      __hip_atomic_store(lc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int i = 0; i < nm; i++) {
        uint64_t *bp = reinterpret_cast<uint64_t *>(a.own + (a.m[i].push ? dm::kBaseSendOff : dm::kBaseRecvOff)) +
                       a.m[i].peer;
        __hip_atomic_store(bp, __hip_atomic_load(bp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// CUs of the current device (0: unknown), queried once per device
static int dm_cus() {
  static std::mutex mu;
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 0;
  }
  std::lock_guard<std::mutex> g(mu);
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    cus[dev] = 0;
  }
  return cus[dev];
}

template <typename T, int OP>
static hipError_t fused_launch(const DmFusedArgs &a0, hipStream_t st) {
  DmFusedArgs a = a0;
  int w = a.wgs;
  dm_fit_residency(&w, 1, nullptr, dm_cap((const void *)k_dm_fused<T, OP>, a.share));
  // above one workgroup per CU, whole multiples of the CU count: every CU
  // carries the same share of every phase (C3 at P = 2 on one GPU: 256 and
  // 512 workgroups 0.41-0.42 ms, 320 / 384 / 640 0.47-0.54 ms)
  const int cus = dm_cus();
  if (cus > 0 && w > cus) w -= w % cus;
  a.wgs = w;
  hipLaunchKernelGGL((k_dm_fused<T, OP>), dim3((unsigned)a.wgs), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

template <typename T>
static hipError_t fused_t(const DmFusedArgs &a, int op, hipStream_t st) {
#define CALL(OP) fused_launch<T, OP>(a, st)
  BINE_OP_SWITCH(T, CALL)
#undef CALL
}

bool dm_fused_supported(int dtype, int op) {
  const bool t = dtype == BINE_FLOAT || dtype == BINE_DOUBLE || dtype == BINE_INT32 || dtype == BINE_INT64 ||
                 dtype == BINE_UINT32 || dtype == BINE_UINT64;
  return t && op >= BINE_SUM && op <= BINE_MIN;
}

int dm_fused_check(const DmFusedArgs &a, int dtype, int op) {
  if (!dm_fused_supported(dtype, op)) return BINE_ERR_UNSUPPORTED;
  const int nm = a.d0 + a.nd;
  if (a.wgs < 1 || !a.own || !a.slot || a.nl < 2 || a.nl > kMaxLeaves || a.pos < 0 || a.pos >= a.nl ||
      a.nt < 1 || a.nt > kMaxFusedTrees || a.na < 0 || a.nd < 0 || nm > kMaxFusedMsgs)
    return BINE_ERR_ARG;
  for (int i = 0; i < nm; i++) {
    const DmMsg &m = a.m[i];
    if (m.peer < 0 || m.peer >= dm::kMaxPeers || m.j < 0 || m.j >= dm::kSlots || m.bytes > a.slot ||
        m.bytes % 16 || ((uintptr_t)(m.push ? (const void *)m.src : (const void *)m.dst) & 15))
      return BINE_ERR_ARG;
  }
  // the layout: A pushes, then each tree's leaf pulls and result pushes, then D pulls
  int at = a.na;
  for (int i = 0; i < a.na; i++)
    if (!a.m[i].push) return BINE_ERR_ARG;
  for (int ti = 0; ti < a.nt; ti++) {
    const DmFusedTree &t = a.t[ti];
    if (t.b0 != at || t.nb != a.nl - 1 || t.nc < 0 || !t.nvec || !t.out || !t.own_leaf ||
        ((uintptr_t)t.out & 15) || ((uintptr_t)t.own_leaf & 15))
      return BINE_ERR_ARG;
    for (int i = t.b0; i < t.b0 + t.nb; i++)
      if (a.m[i].push || a.m[i].bytes != t.nvec * 16) return BINE_ERR_ARG;
    for (int i = t.b0 + t.nb; i < t.b0 + t.nb + t.nc; i++)
      if (!a.m[i].push || a.m[i].bytes != t.nvec * 16) return BINE_ERR_ARG;
    uint32_t seen = 0;
    for (int j = 0; j < a.nl; j++) {
      if (j == a.pos) continue;
      const int i = t.leaf[j];
      if (i < t.b0 || i >= t.b0 + t.nb || (seen >> (i - t.b0) & 1)) return BINE_ERR_ARG;
      seen |= 1u << (i - t.b0);
    }
    at += t.nb + t.nc;
  }
  if (a.d0 != at) return BINE_ERR_ARG;
  for (int i = a.d0; i < nm; i++)
    if (a.m[i].push) return BINE_ERR_ARG;
  return BINE_SUCCESS;
}

int launch_dm_fused(const DmFusedArgs &a, int dtype, int op, void *stream) {
  if (int rc = dm_fused_check(a, dtype, op)) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  switch (dtype) {
    case BINE_FLOAT: e = fused_t<float>(a, op, st); break;
    case BINE_DOUBLE: e = fused_t<double>(a, op, st); break;
    case BINE_INT32: e = fused_t<int32_t>(a, op, st); break;
    case BINE_INT64: e = fused_t<int64_t>(a, op, st); break;
    case BINE_UINT32: e = fused_t<uint32_t>(a, op, st); break;
    case BINE_UINT64: e = fused_t<uint64_t>(a, op, st); break;
    default: return BINE_ERR_UNSUPPORTED;
  }
  return e == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// ----------------------------------------------------------------------------
// cross-GPU flag latency probe (bine_comm_direct_ping).
// One lane of one workgroup on each of two ranks plays ping-pong with the
// transport's own flag protocol -- a relaxed system-scope store of a sequence
// number into the peer's inbox, a relaxed system-scope poll (with the
// protocol's back-off) of the peer's answer in its own -- `iters` times in one
// launch, no kernel boundary in between.  Round trip 1 absorbs the two
// launches' skew; rounds 2 .. iters are timed with wall_clock64 on each side.
// A round trip is two one-way flag latencies: a k_dm_fused phase boundary
// costs one (pico_amd/model.py T_FLAG_US).  Timed out: the transport is
// poisoned like any other wait, *out = 0.
__global__ __launch_bounds__(64) void k_dm_ping(DmPingArgs a) {
  using namespace dm;
  if (threadIdx.x != 0) return;
  uint32_t *poison = reinterpret_cast<uint32_t *>(a.own + kPoisonOff);
  const uint64_t *mine = reinterpret_cast<const uint64_t *>(a.own + kPingOff + (size_t)a.peer * kFlagStride);
  uint8_t *remote = reinterpret_cast<uint8_t *const *>(a.own + kPeerTabOff)[a.peer];
  uint64_t *theirs = reinterpret_cast<uint64_t *>(remote + kPingOff + (size_t)a.rank * kFlagStride);
  if (__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
    __hip_atomic_store(a.out, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  uint64_t t0 = 0;
  for (int i = 1; i <= a.iters; i++) {
    if (i == 2) t0 = wall_clock64();
    const uint64_t s = a.base + (uint64_t)i;
    if (a.initiator) publish(theirs, s);
    const long long w0 = wall_clock64();
    uint64_t seen;
    while ((seen = ld_rlx_sys(mine)) < s) {
      if (wall_clock64() - w0 > (long long)a.timeout_ticks) {
        dm_time_out(poison, a.poison_host, kWaitPing, 0, a.rank, a.peer, 0, s, seen, a.serial, wall_clock64() - w0);
        __hip_atomic_store(a.out, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!a.initiator) publish(theirs, s);
  }
  __hip_atomic_store(a.out, wall_clock64() - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int launch_dm_ping(const DmPingArgs &a, void *stream) {
  if (a.iters < 2 || !a.own || !a.out || a.peer == a.rank) return BINE_ERR_ARG;
  hipLaunchKernelGGL(k_dm_ping, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// ----------------------------------------------------------------------------
// pico_core input generator (glibc rand_r, LCG jump-ahead)
// ----------------------------------------------------------------------------

struct Affine { uint32_t m, c; };  // x -> m x + c (mod 2^32)

__host__ __device__ inline Affine compose(Affine f, Affine g) {  // f(g(x))
  return {f.m * g.m, f.m * g.c + f.c};
}
__host__ __device__ inline Affine lcg_pow(uint64_t k) {
  Affine r{1u, 0u}, p{1103515245u, 12345u};
  while (k) {
    if (k & 1) r = compose(p, r);
    p = compose(p, p);
    k >>= 1;
  }
  return r;
}
// one glibc rand_r() call (three LCG steps, 11+10+10 bits)
__device__ inline int32_t rand_r_step(uint32_t &s) {
  s = s * 1103515245u + 12345u;
  uint32_t r = (s >> 16) % 2048u;
  s = s * 1103515245u + 12345u;
  r = (r << 10) ^ ((s >> 16) % 1024u);
  s = s * 1103515245u + 12345u;
  r = (r << 10) ^ ((s >> 16) % 1024u);
  return (int32_t)r;
}

constexpr int kFillPer = 16;  // consecutive elements per lane

template <typename T, int DT>
__global__ __launch_bounds__(kBlock) void k_fill_pico(T *buf, size_t n, uint32_t seed) {
  constexpr int calls = (DT == BINE_INT64 || DT == BINE_UINT64) ? 2 : 1;
  const size_t first = ((size_t)blockIdx.x * kBlock + threadIdx.x) * kFillPer;
  if (first >= n) return;
  const Affine j = lcg_pow((uint64_t)first * 3u * calls);
  uint32_t s = j.m * seed + j.c;
  for (int k = 0; k < kFillPer && first + k < n; k++) {
    T v;
    if constexpr (DT == BINE_INT8) v = (T)((rand_r_step(s) % 256) - 128);
    else if constexpr (DT == BINE_UINT8) v = (T)(rand_r_step(s) % 256);
    else if constexpr (DT == BINE_INT16) v = (T)((rand_r_step(s) % 65536) - 32768);
    else if constexpr (DT == BINE_UINT16) v = (T)(rand_r_step(s) % 65536);
    else if constexpr (DT == BINE_INT32 || DT == BINE_UINT32) v = (T)rand_r_step(s);
    else if constexpr (DT == BINE_INT64 || DT == BINE_UINT64) {
      const int64_t hi = (int64_t)rand_r_step(s) << 32;
      v = (T)(hi | (int64_t)rand_r_step(s));
    } else if constexpr (DT == BINE_FLOAT) v = (float)rand_r_step(s) / (float)2147483647 * 100.0f;
    else v = (double)rand_r_step(s) / (double)2147483647 * 100.0;
    buf[first + k] = v;
  }
}

int launch_fill_pico(void *buf, size_t n, int dtype, uint32_t seed, void *stream) {
  if (n == 0) return BINE_SUCCESS;
  hipStream_t st = (hipStream_t)stream;
  const size_t lanes = (n + kFillPer - 1) / kFillPer;
  const unsigned blocks = (unsigned)((lanes + kBlock - 1) / kBlock);
#define FILL(T, DT) hipLaunchKernelGGL((k_fill_pico<T, DT>), dim3(blocks), dim3(kBlock), 0, st, (T *)buf, n, seed); break
  switch (dtype) {
    case BINE_INT8: FILL(int8_t, BINE_INT8);
    case BINE_UINT8: FILL(uint8_t, BINE_UINT8);
    case BINE_INT16: FILL(int16_t, BINE_INT16);
    case BINE_UINT16: FILL(uint16_t, BINE_UINT16);
    case BINE_INT32: FILL(int32_t, BINE_INT32);
    case BINE_UINT32: FILL(uint32_t, BINE_UINT32);
    case BINE_INT64: FILL(int64_t, BINE_INT64);
    case BINE_UINT64: FILL(uint64_t, BINE_UINT64);
    case BINE_FLOAT: FILL(float, BINE_FLOAT);
    case BINE_DOUBLE: FILL(double, BINE_DOUBLE);
    default: return BINE_ERR_UNSUPPORTED;
  }
#undef FILL
  return hipGetLastError() == hipSuccess ? BINE_SUCCESS : BINE_ERR_HIP;
}

// ----------------------------------------------------------------------------
// order-independent checksum
// ----------------------------------------------------------------------------

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finalizer
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename U>
__global__ __launch_bounds__(kBlock) void k_checksum(const U *buf, size_t n, unsigned long long *out) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
    acc += mix64((uint64_t)buf[i] + (uint64_t)i * 0x9E3779B97F4A7C15ull);
  // wave64 reduction (two 32-bit shuffles per step)
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)acc, off, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(acc >> 32), off, 64);
    acc += ((uint64_t)hi << 32) | lo;
  }
  __shared__ uint64_t part[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (int w = 0; w < kBlock / 64; w++) s += part[w];
    atomicAdd(out, (unsigned long long)s);
  }
}

int launch_checksum(const void *buf, size_t n, int dtype, uint64_t *host_out, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  unsigned long long *d = nullptr;
  if (hipMalloc(&d, sizeof *d) != hipSuccess) return BINE_ERR_NO_MEM;
  int rc = BINE_SUCCESS;
  if (hipMemsetAsync(d, 0, sizeof *d, st) != hipSuccess) rc = BINE_ERR_HIP;
  size_t blocks = (n + kBlock * 8 - 1) / (kBlock * 8);
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) blocks = 1;
  if (rc == BINE_SUCCESS) {
    switch (bine_dtype_size(dtype)) {
      case 1: hipLaunchKernelGGL((k_checksum<uint8_t>), dim3((unsigned)blocks), dim3(kBlock), 0, st, (const uint8_t *)buf, n, d); break;
      case 2: hipLaunchKernelGGL((k_checksum<uint16_t>), dim3((unsigned)blocks), dim3(kBlock), 0, st, (const uint16_t *)buf, n, d); break;
      case 4: hipLaunchKernelGGL((k_checksum<uint32_t>), dim3((unsigned)blocks), dim3(kBlock), 0, st, (const uint32_t *)buf, n, d); break;
      case 8: hipLaunchKernelGGL((k_checksum<uint64_t>), dim3((unsigned)blocks), dim3(kBlock), 0, st, (const uint64_t *)buf, n, d); break;
      default: rc = BINE_ERR_UNSUPPORTED;
    }
  }
  unsigned long long h = 0;
  if (rc == BINE_SUCCESS && (hipGetLastError() != hipSuccess ||
                             hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st) != hipSuccess ||
                             hipStreamSynchronize(st) != hipSuccess))
    rc = BINE_ERR_HIP;
  (void)hipFree(d);
  if (rc == BINE_SUCCESS) *host_out = h;
  return rc;
}

// workgroup slots of the current device for one direct-transport kernel
// (bine_dm_launch_cap): kind 0 k_dm_move, 1 k_dm_move_tree<T, OP, nl>,
// 2 k_dm_fused<T, OP>; T / OP from (dtype, op) as the launchers pick them
template <typename T>
static const void *dm_kernel_t(int kind, int op, int nl) {
  auto pick = [&](auto opc) -> const void * {
    constexpr int OP = decltype(opc)::value;
    return kind == 1 ? dmt_kernel<T, OP>(nl) : (const void *)k_dm_fused<T, OP>;
  };
  switch (op) {
    case BINE_SUM: return pick(std::integral_constant<int, BINE_SUM>{});
    case BINE_PROD: return pick(std::integral_constant<int, BINE_PROD>{});
    case BINE_MAX: return pick(std::integral_constant<int, BINE_MAX>{});
    case BINE_MIN: return pick(std::integral_constant<int, BINE_MIN>{});
    default: return nullptr;
  }
}

int dm_launch_cap(int kind, int dtype, int op, int nl, int share) {
  const void *k = nullptr;
  if (kind == 0) {
    k = (const void *)k_dm_move;
  } else if (kind == 1 || kind == 2) {
    switch (dtype) {
      case BINE_FLOAT: k = dm_kernel_t<float>(kind, op, nl); break;
      case BINE_DOUBLE: k = dm_kernel_t<double>(kind, op, nl); break;
      case BINE_INT32: k = dm_kernel_t<int32_t>(kind, op, nl); break;
      case BINE_INT64: k = dm_kernel_t<int64_t>(kind, op, nl); break;
      case BINE_UINT32: k = dm_kernel_t<uint32_t>(kind, op, nl); break;
      case BINE_UINT64: k = dm_kernel_t<uint64_t>(kind, op, nl); break;
      default: break;
    }
  }
  return k ? dm_cap(k, share) : -1;
}

}  // namespace bine

extern "C" int bine_set_reduce_tuning(int unroll, int maxblocks, int nontemporal) {
  bine::g_unroll = (unroll == 1 || unroll == 2 || unroll == 4 || unroll == 8) ? unroll : bine::kDefaultUnroll;
  bine::g_maxblocks = maxblocks;
  bine::g_nt = nontemporal;
  return BINE_SUCCESS;
}

#endif  // BINE_OPSET == 0
#if BINE_OPSET != 0
}  // namespace bine
#endif
