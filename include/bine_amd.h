/*
 * bine_amd.h -- core C ABI of the MI355X Bine reduce-family library
 * (libbine_amd.so).  Plain pointers and sizes; no MPI, torch or HIP types in
 * the signatures (HIP streams travel as void*).
 *
 * This is the layer the libbine.h drop-in (include/libbine_amd.h, built as
 * libbine.so) sits on, and the layer Python binds through ctypes.  Every
 * collective entry point replaces one function of the reference's public API
 * (reference include/libbine.h:30-78); the mapping is listed next to each
 * enumerator of bine_algo below.
 *
 * Device pointers only: the buffers passed here must live in the memory of the
 * communicator's device.  Operations are stream-ordered: they are enqueued on
 * `stream` (a hipStream_t; NULL = the HIP null stream, as in HIP and RCCL --
 * pass bine_comm_stream() for the communicator's own) and return once
 * enqueued; a synchronize on `stream` (or bine_comm_synchronize) waits for
 * completion, exchanges included.
 */
#ifndef BINE_AMD_H
#define BINE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types; same numbering as the test oracle (oracle/bine_oracle.h) */
typedef enum {
  BINE_INT8 = 0, BINE_UINT8 = 1, BINE_INT16 = 2, BINE_UINT16 = 3,
  BINE_INT32 = 4, BINE_UINT32 = 5, BINE_INT64 = 6, BINE_UINT64 = 7,
  BINE_FLOAT = 8, BINE_DOUBLE = 9,
  /* MPI's (value, index) pair types, for BINE_MAXLOC / BINE_MINLOC only; C
   * layouts as MPI defines them: FLOAT_INT {float; int} 8 B, DOUBLE_INT
   * {double; int} 16 B, LONG_INT {long; int} 16 B, 2INT {int; int} 8 B,
   * SHORT_INT {short; int} 8 B (padding bytes are never written) */
  BINE_FLOAT_INT = 10, BINE_DOUBLE_INT = 11, BINE_LONG_INT = 12, BINE_2INT = 13, BINE_SHORT_INT = 14,
  /* C99 complex types {re; im} (MPI_C_FLOAT_COMPLEX, MPI_C_DOUBLE_COMPLEX),
   * SUM / PROD only, as MPICH */
  BINE_C_FLOAT_COMPLEX = 15, BINE_C_DOUBLE_COMPLEX = 16,
  BINE_NUM_DTYPES = 17
} bine_dtype_t;

/* reduction operators, MPI_Reduce_local semantics of MPICH 3.3.2:
 * inout[i] = inout[i] (op) in[i]; MAX/MIN select inout when inout > in
 * (resp. <), else in (NaN behaviour follows from that).  The logical ops
 * (MPICH's MPIR_LLAND/LLOR/LLXOR: C truthiness, result 0 or 1 of the element
 * type; defined on every type, floats included -- -0.0 is false, NaN true)
 * and the bitwise ops (integer types only; BINE_ERR_ARG on float / double,
 * where MPICH reports MPI_ERR_OP) complete the predefined MPI_Op set
 * libbine's callers can pass.  MAXLOC / MINLOC (MPICH's opmaxloc.c /
 * opminloc.c: equal values keep the smaller index, otherwise the larger /
 * smaller value's pair; a NaN never replaces nor is replaced) apply to the
 * pair types only, and the pair types to them only. */
typedef enum {
  BINE_SUM = 0, BINE_PROD = 1, BINE_MAX = 2, BINE_MIN = 3,
  BINE_LAND = 4, BINE_BAND = 5, BINE_LOR = 6, BINE_BOR = 7, BINE_LXOR = 8, BINE_BXOR = 9,
  BINE_MAXLOC = 10, BINE_MINLOC = 11,
  BINE_NUM_OPS = 12
} bine_op_t;

typedef enum {
  BINE_SUCCESS = 0,
  BINE_ERR_ARG = 1,          /* reference returns MPI_ERR_ARG (e.g. non-power-of-two remap) */
  BINE_ERR_SIZE = 2,         /* reference returns MPI_ERR_SIZE */
  BINE_ERR_NO_MEM = 3,
  BINE_ERR_HIP = 4,          /* a HIP runtime call failed */
  BINE_ERR_RCCL = 5,         /* an RCCL call failed */
  BINE_ERR_UNSUPPORTED = 6,  /* algorithm / dtype / op not provided */
  BINE_ERR_INTERNAL = 7,
  BINE_ERR_ROOT = 8,         /* reference returns MPI_ERR_ROOT (bcast_bine_lat: root != 0) */
  BINE_ERR_COUNT = 9         /* reference returns MPI_ERR_COUNT (bandwidth bcasts: count < P) */
} bine_status_t;

/* Algorithms.  Names are the libbine function names without the collective
 * prefix; bine_algo_from_name() also accepts the full function name and the
 * pico_core selector strings (pico_core_utils.c:103-249, e.g.
 * "bine_bdw_remap_over"). */
typedef enum {
  /* allreduce_* -- libbine_allreduce.c */
  BINE_AR_RECURSIVEDOUBLING = 0,      /* allreduce_recursivedoubling      :17   */
  BINE_AR_RING = 1,                   /* allreduce_ring                   :138  */
  BINE_AR_RABENSEIFNER = 2,           /* allreduce_rabenseifner           :441  */
  BINE_AR_BINE_LAT = 3,               /* allreduce_bine_lat               :321  */
  BINE_AR_BINE_BDW_STATIC = 4,        /* allreduce_bine_bdw_static        :696  */
  BINE_AR_BINE_BDW_REMAP = 5,         /* allreduce_bine_bdw_remap         :820  */
  BINE_AR_BINE_BDW_REMAP_SEGMENTED = 6, /* allreduce_bine_bdw_remap_segmented :1093 */
  BINE_AR_BINE_BLOCK_BY_BLOCK_ANY_EVEN = 7, /* allreduce_bine_block_by_block_any_even :925 */
  /* reduce_scatter_* -- libbine_reduce_scatter.c */
  BINE_RS_RECURSIVEHALVING = 16,      /* :15   */
  BINE_RS_RECURSIVE_DISTANCE_DOUBLING = 17, /* :259 */
  BINE_RS_RING = 18,                  /* :421  */
  BINE_RS_BUTTERFLY = 19,             /* :575  */
  BINE_RS_BINE_STATIC = 20,           /* :763  */
  BINE_RS_BINE_SEND_REMAP = 21,       /* :906  */
  BINE_RS_BINE_PERMUTE_REMAP = 22,    /* :985  */
  BINE_RS_BINE_BLOCK_BY_BLOCK = 23,   /* :1066 */
  BINE_RS_BINE_BLOCK_BY_BLOCK_ANY_EVEN = 24, /* :1176 */
  /* reduce_* -- libbine_reduce.c */
  BINE_RD_BINE_LAT = 32,              /* reduce_bine_lat :16 */
  BINE_RD_BINE_BDW = 33,              /* reduce_bine_bdw :83 */
  /* allgather, libbine_allgather.c */
  BINE_AG_RECURSIVEDOUBLING = 48,     /* :18   */
  BINE_AG_K_BRUCK = 49,               /* :88   */
  BINE_AG_RING = 50,                  /* :213  */
  BINE_AG_SPARBIT = 51,               /* :327  */
  BINE_AG_BINE_BLOCK_BY_BLOCK = 52,   /* :410  */
  BINE_AG_BINE_BLOCK_BY_BLOCK_ANY_EVEN = 53, /* :492 */
  BINE_AG_BINE_PERMUTE_STATIC = 54,   /* :563  */
  BINE_AG_BINE_SEND_STATIC = 55,      /* :642  */
  BINE_AG_BINE_PERMUTE_REMAP = 56,    /* :725  */
  BINE_AG_BINE_SEND_REMAP = 57,       /* :811  */
  BINE_AG_BINE_2_BLOCKS = 58,         /* :892  */
  BINE_AG_BINE_2_BLOCKS_DTYPE = 59,   /* :999  */
  /* bcast, libbine_bcast.c (widening past section 8):
   * the latency trees and the scatter + allgather bandwidth variants */
  BINE_BC_SCATTER_ALLGATHER = 64,     /* :42   */
  BINE_BC_BINE_LAT = 65,              /* :189  */
  BINE_BC_BINE_LAT_REVERSED = 66,     /* :281  */
  BINE_BC_BINE_LAT_NEW = 67,          /* :373  */
  BINE_BC_BINE_LAT_I_NEW = 68,        /* :408  */
  BINE_BC_BINE_BDW_STATIC = 69,       /* :462  */
  BINE_BC_BINE_BDW_REMAP = 70,        /* :649  */
  /* alltoall / gather / scatter: whole-block data
   * movement; the plan refuses (BINE_ERR_ROOT at a power-of-two P, else
   * BINE_ERR_SIZE) the (P, root) pairs at which the reference hangs, crashes
   * or delivers a wrong result, and MPI_IN_PLACE (BINE_ERR_ARG) */
  BINE_A2A_BINE = 80,                 /* alltoall_bine libbine_alltoall.c:14 */
  BINE_GA_BINE = 81,                  /* gather_bine   libbine_gather.c:16   */
  BINE_SC_BINE = 82                   /* scatter_bine  libbine_scatter.c:14  */
} bine_algo_t;

/* the reference's MPI_IN_PLACE (mpi.h: (void *)-1) */
#define BINE_IN_PLACE ((const void *)(intptr_t)-1)

typedef struct bine_comm *bine_comm_t;

const char *bine_status_string(int status);
/* text of the last HIP/RCCL failure seen by this thread */
const char *bine_last_error(void);
/* reduce-kernel launch shape (tuning; also env BINE_REDUCE_UNROLL /
 * BINE_REDUCE_MAXBLOCKS / BINE_REDUCE_NT): 16-B vectors in flight per lane
 * (1, 2, 4, 8), grid cap (0 = 2048), non-temporal loads of `in` (fp32 SUM only) */
int bine_set_reduce_tuning(int unroll, int maxblocks, int nontemporal);
size_t bine_dtype_size(int dtype);
/* 1 if MPICH's MPI_Reduce_local accepts (dtype, op): no bitwise op on float /
 * double, MAXLOC / MINLOC exactly on the pair types, SUM / PROD only on the
 * complex types; 0 otherwise (the collectives then return BINE_ERR_ARG, the
 * libbine.h shim MPI_ERR_OP) */
int bine_op_valid(int dtype, int op);
/* -1 if unknown; `collective` = "allreduce" | "reduce_scatter" | "reduce" */
int bine_algo_from_name(const char *collective, const char *name);
const char *bine_algo_name(int algo);

/* ---- the arithmetic boundary: MPI_Reduce_local on the GPU ------------------
 * inout[i] = inout[i] (op) in[i]  (replaces every MPI_Reduce_local call site,
 * e.g. libbine_allreduce.c:888).  `stream` is a hipStream_t (NULL = default). */
int bine_reduce_local(const void *in, void *inout, size_t count, int dtype, int op, void *stream);
/* out[i] = b[i] (op) a[i]  (out may alias b): the copy-free form used for the
 * first step of a non-in-place collective. */
int bine_reduce3(const void *a, const void *b, void *out, size_t count, int dtype, int op, void *stream);

/* pico_core's input distribution (pico_core_utils.c:902-923) generated on the
 * device: element i of buffer `seed` equals what glibc rand_r(&seed) would
 * produce for pico_core (LCG jump-ahead, bit-exact). */
/* n (1..8) independent reductions out[k] = b[k] (op) a[k] in one launch
 * (BINE_ERR_ARG if some window's operands are not co-aligned mod 16 B). */
int bine_reduce_batch(int n, const void *const *a, const void *const *b, void *const *out,
                      const size_t *count, int dtype, int op, void *stream);
/* The owner's side of the flat reduce-scatter (bine_comm_set_flat_rs): out =
 * the binary reduction tree over `nleaves` (2, 4, 8 or 16) blocks given in tree
 * order, evaluated level by level -- v[i] = v[i] (op) v[i + w] for w = 1, 2,
 * 4, ... and i a multiple of 2w (v[i] the inout side) -- in one pass over the
 * operands.  `out` may alias any leaf element for element. */
int bine_reduce_tree(int nleaves, const void *const *leaves, void *out, size_t count, int dtype, int op,
                     void *stream);
int bine_fill_pico(void *buf, size_t count, int dtype, uint32_t seed, void *stream);
/* copy_buffer on the device (libbine_utils.h:176-190; the sbuf -> rbuf copy of
 * e.g. allreduce_bine_bdw_remap, libbine_allreduce.c:849-852): dst[0:bytes) =
 * src[0:bytes), stream-ordered, the kernel every COPY primitive runs. */
int bine_copy(void *dst, const void *src, size_t bytes, void *stream);
/* Order-independent 64-bit digest of a buffer: sum over i of
 * mix64(bits(x[i]) + i * 0x9E3779B97F4A7C15) mod 2^64 (bits zero-extended).
 * Result written to *out (host pointer) after an internal synchronize. */
int bine_checksum(const void *buf, size_t count, int dtype, uint64_t *out, void *stream);

/* ---- communicators ---------------------------------------------------------- */
#define BINE_UNIQUE_ID_BYTES 128
int bine_get_unique_id(void *id /* BINE_UNIQUE_ID_BYTES */);
/* RCCL version codes (NCCL_VERSION encoding, e.g. 22606 = 2.26.6): the library
 * the process maps (ncclGetVersion) and the headers this library was compiled
 * against.  A pure reporter (BINE_ERR_RCCL only when the runtime cannot be
 * asked): whether the pair lies in the window whose ABI for every RCCL type
 * this library passes was checked is bine_rccl_abi_check's answer;
 * bine_comm_init_rccl refuses a pair outside it, and also a runtime whose
 * results in the creation-time ABI probe (every type / op this library
 * passes, run through the runtime) differ. */
int bine_rccl_version(int *runtime, int *compiled);
/* The pure check behind bine_rccl_version: BINE_SUCCESS iff both version codes
 * lie in the checked ABI window (2.26.0 ... 2.27.99). */
int bine_rccl_abi_check(int runtime, int compiled);
/* One process per GPU, RCCL P2P over xGMI.  `id` from rank 0's
 * bine_get_unique_id(), broadcast by the caller (MPI, torch.distributed...). */
int bine_comm_init_rccl(bine_comm_t *comm, int nranks, int rank, const void *id, int device);
/* nranks virtual ranks on ONE device inside this process (in-process peer
 * copies instead of RCCL).  Each rank must be driven from its own host thread
 * (see bine_loopback_run_* below for a ready-made driver). */
int bine_comm_init_loopback(bine_comm_t *comms /* [nranks] */, int nranks, int device);
int bine_comm_destroy(bine_comm_t comm);
int bine_comm_rank(bine_comm_t comm);
int bine_comm_size(bine_comm_t comm);
int bine_comm_device(bine_comm_t comm);
void *bine_comm_stream(bine_comm_t comm);
int bine_comm_synchronize(bine_comm_t comm);

/* Multi-link relay for permutation steps (every rank sends one block to one
 * peer): each pipelining chunk is split into a direct part and P-2 parts that
 * travel two hops through the other ranks, so one step loads every xGMI link
 * instead of one.  Results are unchanged bit for bit (only routes differ).
 * min_part_bytes = smallest relayed part (chunks smaller than P times this go
 * direct); 0 = off (default unless BINE_RELAY_MIN_BYTES is set).  Collective:
 * every rank of the communicator must use the same setting. */
int bine_comm_set_relay(bine_comm_t comm, size_t min_part_bytes);

/* Multi-tree mode for allreduce at P = 4 and 8: the buffer is cut into P-1
 * slices and the algorithm runs once per slice with the ranks relabelled so
 * that at every step the P-1 instances use P-1 edge-disjoint pairings -- all
 * links of the node, one hop each.  Integer results are identical to the
 * reference; floating-point results equal the reference's schedule applied to
 * relabelled ranks (a different association order: within rounding of the
 * reference, not bit-identical).  Off by default (BINE_TREES=1 turns it on);
 * collective: every rank must use the same setting. */
int bine_comm_set_trees(bine_comm_t comm, int on);

/* Pipelining chunk of this communicator's exchanges, in bytes: every step
 * whose received block feeds a reduction is cut into chunks of this size so
 * that chunk k+1's transfer overlaps chunk k's reduction (the device form of
 * the segmented variant's Irecv/Reduce_local loop, libbine_allreduce.c:
 * 1218-1253).  0 = the default (16 MiB, or BINE_CHUNK_BYTES).  Never changes a
 * result bit.  A nonzero `segsize` argument of bine_allreduce still wins for
 * that call.  Collective: every rank must use the same setting. */
int bine_comm_set_chunk(bine_comm_t comm, size_t bytes);

/* Flat allgather phase for allreduce_bine_bdw_remap / _static /
 * _remap_segmented / allreduce_rabenseifner at power-of-two P (and a flat
 * gather for reduce_bine_bdw: every rank sends its reduced block straight to
 * the root): after the reduce-scatter (unchanged,
 * so every reduction sees the reference's operands in the reference's order)
 * every rank sends its reduced block to all other ranks in ONE exchange,
 * instead of the log2(P) mirrored steps (libbine_allreduce.c:779-809,
 * :898-906).  On a fully connected node that is one hop on every link at once.
 * The allgather family (out of place) becomes one all-peers exchange after
 * its own plan has decided the status.  Pure data movement: results
 * identical bit for bit.  Off by default in the core (the literal schedule;
 * BINE_FLAT_AG=1 turns it on; libbine.so turns it on, bine_dropin_defaults);
 * collective.  on = 2 (BINE_FLAT_AG=2): with
 * the flat reduce-scatter too, the allreduces' allgather is cut with the
 * reduce-scatter's chunks, chunk k's results leaving right after chunk k+1's
 * reduce-scatter exchange, so the output completes chunk by chunk. */
int bine_comm_set_flat_ag(bine_comm_t comm, int on);

/* Host-buffer collectives with the host<->device staging pipelined into the
 * collective (libbine.so's path for pico_core's host buffers,
 * pico_core_allreduce_utils.c:13-25).  `host_sbuf` / `host_rbuf` are host
 * memory (page-locked for the copies to be asynchronous), `dev_sbuf` /
 * `dev_rbuf` their device counterparts (workspaces of the same sizes).
 * host_sbuf = BINE_IN_PLACE: in place, the input is host_rbuf (dev_sbuf
 * unused).  The input is copied host -> device piece by piece on `h2d_stream`,
 * each piece just before the first operation that touches it, and the output
 * device -> host on `d2h_stream` piece by piece, each right after the
 * operation that writes it last; the collective runs on `stream` (and the
 * communicator's comm stream), which ends after the last copy back, so
 * synchronizing `stream` completes the call.  For this call the flat forms
 * are on (bine_comm_set_flat_rs, bine_comm_set_flat_ag(2)) where the algorithm
 * has them: the same result bits as the reference (block ownership and every
 * reduction tree follow the whole count, whatever the chunking), while the
 * output completes chunk by chunk, so the two PCIe directions overlap each
 * other and the exchanges.  `chunk_bytes` = bytes one exchange round carries
 * over all blocks (0: 16 MiB).  Never graph-captured.  A NULL `host_sbuf` /
 * `host_rbuf` means that buffer is already on the device: `dev_sbuf` /
 * `dev_rbuf` is the caller's own and nothing is copied for it (its stream
 * argument may then be NULL).  The schedule is the same either way, so ranks
 * with host buffers and ranks with device buffers can meet in one call. */
int bine_allreduce_staged(bine_comm_t comm, int algo, const void *host_sbuf, void *host_rbuf, void *dev_sbuf,
                          void *dev_rbuf, size_t count, int dtype, int op, size_t segsize, size_t chunk_bytes,
                          void *h2d_stream, void *d2h_stream, void *stream);
int bine_reduce_scatter_staged(bine_comm_t comm, int algo, const void *host_sbuf, void *host_rbuf,
                               void *dev_sbuf, void *dev_rbuf, const int *rcounts, int dtype, int op,
                               size_t chunk_bytes, void *h2d_stream, void *d2h_stream, void *stream);

/* Transport option for RCCL communicators (P >= 3): an exchange in which
 * every rank sends ONE buffer to all P-1 others and receives one message of
 * the same size from each -- the flat allgather phase, the one-shot form of
 * allreduce_bine_lat, the allgather family's flat form -- runs as RCCL's
 * ncclAllGather into a staging area followed by P-1 device copies to the
 * receive locations, instead of P-1 ncclSend/ncclRecv pairs.  The same bytes
 * land in the same places (results unchanged); whether RCCL's collective
 * kernels move them faster than its point-to-point path on a given node is
 * measured by bench.py.  The decision is local to each rank but the same on
 * every rank for the plans of this library; a caller of bine_exchange with
 * this option on must keep that shape symmetric too.  Off by default
 * (BINE_COLL_AG=1 turns it on); loopback: BINE_ERR_UNSUPPORTED. */
int bine_comm_set_coll_ag(bine_comm_t comm, int on);

/* Transport option for RCCL communicators (P >= 3), used only with relay and
 * multi-tree mode off: an exchange with exactly one message of the same size
 * to and from every other rank (the flat reduce-scatter and allgather phases)
 * runs as ONE ncclAllToAllv call instead of P-1 ncclSend/ncclRecv pairs; same
 * bytes, same places, results unchanged.  RCCL 2.26 implements ncclAllToAllv
 * with the same grouped point-to-point kernel (rcclGenericKernel, one launch
 * per exchange either way: profiles/r2_a2a_vs_p2p_kernels.txt), so this is an
 * API variant, not a different data path; bench.py no longer trials it.
 * Takes precedence over bine_comm_set_coll_ag.  Off by default
 * (BINE_COLL_A2A=1); collective; loopback: BINE_ERR_UNSUPPORTED. */
int bine_comm_set_coll_a2a(bine_comm_t comm, int on);

/* Flat reduce-scatter phase for every reduce-family algorithm at
 * power-of-two P <= 16 (the rings: the same exchange, their chain folded by
 * P-1 pairwise reductions, since a chain is not a balanced tree): allreduce_bine_bdw_remap / _static /
 * _remap_segmented / _block_by_block_any_even / allreduce_rabenseifner,
 * reduce_scatter_bine_permute_remap / _send_remap / _static / _block_by_block /
 * _block_by_block_any_even / _recursivehalving / _recursive_distance_doubling /
 * _butterfly, reduce_bine_bdw, reduce_bine_lat (every rank's vector straight to
 * the root, the root evaluates the binomial tree), allreduce_bine_lat and
 * allreduce_recursivedoubling (one-shot: every rank's vector to every other,
 * each rank evaluates its own recursive-doubling tree): the log2(P) halving steps
 * become ONE exchange in which every rank sends each block straight to the
 * rank that computes it (one hop on every link at once), and that rank
 * evaluates the reference's reduction tree for its block -- the same binary
 * tree over the same P contributions, same association, same operand order
 * (T(x,s) = T(x,s-1) (op) T(peer(x,s),s-1)) -- in one fused kernel
 * (BINE_PRIM_REDUCE_TREE: reads P blocks, writes one).  Results identical bit
 * for bit to the literal schedule.  Chunked like the other pipelined steps
 * (the transfer of chunk k+1 overlaps the tree of chunk k).  Off by default
 * in the core (BINE_FLAT_RS=1 turns it on; libbine.so turns it on,
 * bine_dropin_defaults); collective. */
int bine_comm_set_flat_rs(bine_comm_t comm, int on);
/* The forms libbine.so (the libbine.h drop-in) gives each communicator it
 * creates for the unchanged pico_core, host only, from
 * the environment at the call: by default the fastest bit-identical forms --
 * the flat reduce-scatter and flat allgather phases (the planner applies them
 * where they exist: power-of-two P, the Bine remap / static / rabenseifner
 * allreduces, the remap / static reduce-scatters, reduce_bine_bdw, the
 * one-shot latency forms; elsewhere the literal schedule) and, at P > 1, the
 * direct peer-memory transport (its fused trees and, where a call's plan fits,
 * the whole call as ONE k_dm_fused launch -- C1 and C3 do); a communicator
 * whose ranks cannot set the direct transport up keeps RCCL P2P.
 * BINE_LITERAL=1: the reference's literal schedule over RCCL P2P (all three
 * off).  BINE_FLAT_RS, BINE_FLAT_AG (0 / 1 / 2) and BINE_DIRECT (0 / 1)
 * override one setting each.  The choice depends on P and the environment
 * only -- the same on every rank. */
int bine_dropin_defaults(int P, int *flat_rs, int *flat_ag, int *direct);

/* Direct peer-memory transport (RCCL communicators, one node): exchanges
 * move through device memory every rank maps from every peer (VMM
 * allocations exported as POSIX file descriptors and handed over Unix
 * sockets; on one node peer memory is reachable over xGMI by plain loads and
 * stores) instead of RCCL's send/receive: each exchange round pushes every
 * outgoing message into one of the receiver's 4 slots for this sender and
 * pulls every incoming message out of its own (a one-round exchange is one
 * kernel launch; longer ones pipeline a round's pulls with the next round's
 * pushes), with release/acquire flags at
 * system scope.  Same bytes in the same places: results bit-identical.  Every
 * wait has a time limit (BINE_DIRECT_TIMEOUT_S, default 10 s); a timeout
 * disables the transport (BINE_ERR_INTERNAL from then on) instead of
 * hanging.  Every call with on = 1 is collective (every rank of the
 * communicator, at the same point): the first sets the transport up, later
 * ones rebuild it on every rank when it was disabled by a timeout on any
 * rank.  Sequence numbers live in device memory,
 * so graph mode captures and replays these collectives too.  At most 4
 * messages to one peer per exchange group
 * (BINE_ERR_UNSUPPORTED beyond).  Knobs: BINE_DIRECT_SLOT_BYTES (64 MiB),
 * BINE_DIRECT_WGS (workgroups per message, 128), BINE_DIRECT_MERGE (launch
 * structure: 3 = the mix above, 2 = one launch per round, 1 = pipelined, 0 =
 * separate push and pull launches).  At most 64 ranks.  Loopback:
 * UNSUPPORTED.  Memory: each rank reserves one inbox of 320 KiB of flags +
 * P x 4 slots x BINE_DIRECT_SLOT_BYTES (64 MiB default: 2 GiB at P = 8,
 * 16 GiB at the 64-rank limit) at set-up, whatever the message sizes; set
 * BINE_DIRECT_SLOT_BYTES lower for small messages or many ranks (a slot
 * below the pipelining chunk only adds launch rounds).  Every launch's
 * workgroups are cut to the GPU's resident capacity divided by the ranks
 * sharing it (bine_dm_launch_cap). */
int bine_comm_set_direct(bine_comm_t comm, int on);
/* Workgroups per message of the direct transport's copy launches (0: the
 * default, BINE_DIRECT_WGS or 128).  Local, not collective; drops cached graphs
 * (their launches carry the old grid).  bench.py trials it on the node. */
int bine_comm_set_direct_wgs(bine_comm_t comm, int wgs);
/* Direct transport: the flat reduce-scatter's trees evaluated inside the
 * exchange launches (on >= 1: the leaves read in place in the inbox slots,
 * each tree in the first launch of the exchange after the one that receives
 * its leaves, or in its own -- the default; on >= 2 also sets the tree
 * workgroups per launch (1: BINE_DIRECT_TREE_WGS, 256); 0: pull copies into
 * the staging area + a separate tree launch; -1: BINE_DIRECT_TREE, default
 * on).  Bit-identical either way.  Collective: every rank must use the same
 * setting (it decides in which launch a leaf is pulled).  Local call; drops
 * cached graphs.  bench.py trials it on the node ("+dm" vs "+dmt"
 * transports, "+dmtxT" for T tree workgroups). */
int bine_comm_set_direct_tree(bine_comm_t comm, int on);
/* Diagnostics of the direct transport (BINE_DIRECT_STAMPS=<records> in the
 * environment when the transport is set up): every workgroup of every
 * exchange launch appends one record of 4 words -- tag = launch serial << 32
 * | kind << 24 | message << 16 | workgroup (kind 0 push, 1 pull, 2 tree), and
 * its wall_clock64 at entry, when its wait ended and when its copy or tree
 * ended.  Copies up to `cap` records into `out` (4 words each) after
 * synchronizing the device, sets *n to the number written so far (may exceed
 * cap), and with reset != 0 starts over.  BINE_ERR_UNSUPPORTED when stamps are
 * off. */
int bine_comm_direct_stamps(bine_comm_t comm, uint64_t *out, size_t cap, size_t *n, int reset);
/* 1 when a wait of this rank's direct transport timed out (the transport is
 * disabled until the next collective bine_comm_set_direct(1) rebuilds it;
 * a call in flight at that moment completed without its data), 0 otherwise
 * or without a direct transport; -status on error.  Host-only read of the
 * mapped poison word: call it after synchronizing. */
int bine_comm_direct_timed_out(bine_comm_t comm);
/* Cross-GPU flag latency of the direct transport: this
 * rank and `peer` play `iters` (>= 2) flag round trips with the transport's
 * own protocol -- a system-scope store into the peer's inbox, a poll of its
 * answer in ours -- inside ONE launch on each side, no kernel boundary in
 * between; *us = microseconds per round trip over round trips 2 .. iters as
 * this rank's clock saw them (the lower rank starts each round trip).  BOTH
 * ranks of the pair must call it together, after the communicator's earlier
 * work (it synchronizes the communicator's streams first and blocks until
 * done).  A timed-out wait poisons the transport as any other
 * (BINE_ERR_INTERNAL); BINE_ERR_UNSUPPORTED without a direct transport. */
int bine_comm_direct_ping(bine_comm_t comm, int peer, int iters, double *us);

/* Graph mode (RCCL communicators): the first collective call for a given
 * (algorithm, arguments, buffers, dtype, op, stream) captures the whole issue
 * sequence -- RCCL's grouped P2P launches on the comm stream, the reduction
 * kernels on the caller's stream and the event hand-offs between them -- into
 * one HIP graph; every later call with the same key replays it with one
 * hipGraphLaunch, so the host issue cost of a collective is one launch.
 * Same work, same order: results bit-identical.  The caller's stream must not
 * be the NULL stream (not capturable; such calls run eagerly), and buffers
 * must stay allocated while their graph is cached (up to 64 graphs; the cache
 * is dropped when the workspace grows and when graph mode is switched off).
 * Schedules on two streams (graphs with parallel branches) are captured only
 * on HIP runtimes >= 7.2; on older ones (torch's bundled 7.0) they run
 * eagerly: that runtime's hipGraphLaunch crashes on such graphs when their
 * streams share one hardware queue (tools/graph_fork_repro.cpp).  RCCL forks
 * streams of its own inside a capture, so on such a runtime single-stream
 * calls are captured over the direct transport with GPU_MAX_HW_QUEUES >= 2
 * and over RCCL with >= 4 (HIP's default); the rest runs eagerly.
 * Off by default (BINE_GRAPHS=1 turns it on); loopback: BINE_ERR_UNSUPPORTED. */
int bine_comm_set_graphs(bine_comm_t comm, int on);
/* Number of graphs graph mode holds (captured and replayable) -- 0 while
 * every call ran eagerly (graph mode off, NULL stream, or a schedule the
 * runtime gate above keeps eager); -status on error. */
int64_t bine_comm_graphs_cached(bine_comm_t comm);
/* Large collectives this communicator issued as ONE k_dm_fused launch over
 * the direct transport (every exchange and tree of the call in one kernel:
 * bine_comm_set_direct + bine_comm_set_direct_tree on, flat phases, at most
 * 4 slot-sized chunks; BINE_DIRECT_FUSED_LARGE=0 turns the form off);
 * eager issues only (graph replays are not counted). */
int64_t bine_comm_fused_calls(bine_comm_t comm);

/* Per-op device timing ("hipEvents per step"): with profiling on, every op
 * of a collective's issue schedule -- an exchange group on the comm stream or
 * a local primitive on the caller's stream -- is bracketed by two timing
 * events on its stream (single-stream small collectives: all on the caller's
 * stream).
 * bine_comm_profile() waits for the latest collective's events and fills one
 * entry per op: kind, primitives, bytes (exchange: bytes this rank sends;
 * local: algorithmic HBM bytes), start relative to the first op's start and
 * duration.  An op evaluated inside another exchange's launch (the direct
 * transport's fused trees) reports nprims = 0, bytes = 0 and ~0 ms: its time
 * is the hosting exchange's.  Returns the number of ops (may exceed cap) or
 * -status.  Off by default (the events cost host time per op).  BINE_ROCTX=1 additionally
 * brackets every collective and every issued op with a roctx range. */
typedef struct {
  int32_t xchg;
  int32_t nprims;
  uint64_t bytes;
  float start_ms;
  float ms;
} bine_op_time_t;
int bine_comm_set_profile(bine_comm_t comm, int on);
int64_t bine_comm_profile(bine_comm_t comm, bine_op_time_t *out, int64_t cap);

/* ---- collectives (device pointers, stream-ordered) ------------------------- */
/* allreduce_* (libbine.h:30-37).  `segsize` plays bine_allreduce_segsize
 * (libbine.h:28) for BINE_AR_BINE_BDW_REMAP_SEGMENTED and is the pipelining
 * chunk of the other bandwidth variants (0 = library default). */
int bine_allreduce(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count,
                   int dtype, int op, size_t segsize, void *stream);
/* reduce_scatter_* (libbine.h:69-77) */
int bine_reduce_scatter(bine_comm_t comm, int algo, const void *sbuf, void *rbuf,
                        const int *rcounts, int dtype, int op, void *stream);
/* reduce_* (libbine.h:64-65).  rbuf is only read on `root` (may be NULL elsewhere). */
int bine_reduce(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count,
                int dtype, int op, int root, void *stream);
/* allgather_* (libbine.h:39-50), scount = rcount = `count` elements per rank of
 * one type (as pico_core calls them, pico_core_utils.c:511-514); rbuf holds
 * nranks * count elements.  sbuf = BINE_IN_PLACE follows the reference: rank
 * r's block is expected where that algorithm's in-place path expects it (block
 * r; block perm[r] / remap[r] for the permute variants); the send and
 * any_even variants have no in-place path (BINE_ERR_ARG). */
int bine_allgather(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count,
                   int dtype, void *stream);
/* bcast_* (libbine.h:54-60): `buf` (count elements) of `root` reaches every
 * rank, whole-buffer transfers along the algorithm's tree.  Power-of-two P
 * only (BINE_ERR_SIZE otherwise); bine_lat / bine_lat_reversed take root 0
 * only (BINE_ERR_ROOT), as the reference. */
int bine_bcast(bine_comm_t comm, int algo, void *buf, size_t count, int dtype, int root, void *stream);
/* gather_bine / scatter_bine / alltoall_bine (libbine.h:52, :63, :78; sendcount
 * = recvcount = `count` elements per block, one type).  gather: sbuf `count`
 * elements on every rank, rbuf P * count on the root (unused elsewhere, may be
 * NULL); scatter: sbuf P * count on the root (unused elsewhere, may be NULL),
 * rbuf `count`; alltoall: sbuf and rbuf P * count, block j of sbuf goes to
 * rank j.  Pure data movement.  The literal schedules of the reference, or
 * with bine_comm_set_flat_ag(1) one direct exchange (every block straight to
 * its destination); refused (BINE_ERR_ROOT / BINE_ERR_SIZE) where the
 * reference does not deliver the collective, BINE_ERR_ARG for MPI_IN_PLACE. */
int bine_gather(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int root,
                void *stream);
int bine_scatter(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, int root,
                 void *stream);
int bine_alltoall(bine_comm_t comm, int algo, const void *sbuf, void *rbuf, size_t count, int dtype, void *stream);

/* One group of point-to-point transfers on the communicator's transport (RCCL:
 * ncclSend / ncclRecv inside one ncclGroupStart/End) -- the MPI_Sendrecv /
 * Isend+Irecv+Waitall building block of every libbine schedule
 * (e.g. libbine_allreduce.c:866-870), exposed for link calibration
 * (bench.py's RCCL P2P probe) and tests.  Byte counts; receives must match the
 * peers' sends in count and posting order.  Stream-ordered like the
 * collectives (runs after the caller's prior work on `stream`, which waits for
 * it).  RCCL communicators only (loopback: BINE_ERR_UNSUPPORTED). */
int bine_exchange(bine_comm_t comm, int nsend, const int *send_peers, const void *const *sbufs,
                  const size_t *sbytes, int nrecv, const int *recv_peers, void *const *rbufs,
                  const size_t *rbytes, void *stream);

/* RCCL's own ncclAllReduce on the communicator's RCCL communicator -- the
 * vendor collective, NOT a libbine algorithm (its reduction order is RCCL's,
 * so fp results are not the reference's bits).  A measurement baseline only:
 * bench.py times it beside the Bine path on the same node, buffers and
 * stream ordering.  RCCL communicators only (loopback: BINE_ERR_UNSUPPORTED). */
int bine_vendor_allreduce(bine_comm_t comm, const void *sbuf, void *rbuf, size_t count, int dtype,
                          int op, void *stream);

/* ---- loopback drivers: run one collective on all virtual ranks ---------------
 * (one host thread per rank; returns the first non-success status) */
int bine_loopback_run_allreduce(bine_comm_t *comms, int nranks, int algo,
                                const void *const *sbufs, void *const *rbufs, size_t count,
                                int dtype, int op, size_t segsize, int *statuses);
int bine_loopback_run_reduce_scatter(bine_comm_t *comms, int nranks, int algo,
                                     const void *const *sbufs, void *const *rbufs,
                                     const int *rcounts, int dtype, int op, int *statuses);
int bine_loopback_run_reduce(bine_comm_t *comms, int nranks, int algo,
                             const void *const *sbufs, void *const *rbufs, size_t count,
                             int dtype, int op, int root, int *statuses);
int bine_loopback_run_allgather(bine_comm_t *comms, int nranks, int algo,
                                const void *const *sbufs, void *const *rbufs, size_t count,
                                int dtype, int *statuses);
int bine_loopback_run_bcast(bine_comm_t *comms, int nranks, int algo, void *const *bufs,
                            size_t count, int dtype, int root, int *statuses);
int bine_loopback_run_gather(bine_comm_t *comms, int nranks, int algo, const void *const *sbufs,
                             void *const *rbufs, size_t count, int dtype, int root, int *statuses);
int bine_loopback_run_scatter(bine_comm_t *comms, int nranks, int algo, const void *const *sbufs,
                              void *const *rbufs, size_t count, int dtype, int root, int *statuses);
int bine_loopback_run_alltoall(bine_comm_t *comms, int nranks, int algo, const void *const *sbufs,
                               void *const *rbufs, size_t count, int dtype, int *statuses);

/* ---- schedule introspection (host only, no GPU needed) ----------------------
 * A plan is the ordered list of primitives one rank executes. */
typedef enum { BINE_PRIM_SEND = 1, BINE_PRIM_RECV = 2, BINE_PRIM_REDUCE = 3,
               BINE_PRIM_REDUCE3 = 4, BINE_PRIM_COPY = 5,
               BINE_PRIM_REDUCE_TREE = 6  /* flat reduce-scatter: see bine_comm_set_flat_rs */
} bine_prim_type_t;
typedef enum { BINE_BUF_SBUF = 0, BINE_BUF_RBUF = 1, BINE_BUF_TMP0 = 2, BINE_BUF_TMP1 = 3,
               BINE_BUF_TMP2 = 4,
               BINE_BUF_STAGE = 5  /* relay staging; appears in issue schedules only */
} bine_buf_t;
#define BINE_PRIM_PIPELINE 1  /* flags: exchange whose receive feeds the next
                                 REDUCE(3) element for element -- both may be
                                 split into chunks and overlapped */
/* REDUCE_TREE: flags >> 8 = levels whose combine is v[i + w] (op) v[i] (the
   right subtree is the inout side; block_by_block's last step) */
typedef struct {
  int32_t type;      /* bine_prim_type_t */
  int32_t group;     /* consecutive SEND/RECV with equal group form one exchange */
  int32_t peer;      /* SEND/RECV peer rank; REDUCE_TREE: number of leaves nl */
  int32_t flags;     /* BINE_PRIM_PIPELINE */
  int32_t src_buf;   /* SEND: source; REDUCE/REDUCE3: `in` (a); COPY: source;
                        REDUCE_TREE: the other nl-1 leaves, k-th at src_off + k*count */
  int32_t dst_buf;   /* RECV: destination; REDUCE: inout; REDUCE3 / REDUCE_TREE: out; COPY: dest */
  int32_t aux_buf;   /* REDUCE3: b; REDUCE_TREE: the rank's own leaf (position `pos`) */
  int32_t pos;       /* REDUCE_TREE: tree position of the aux leaf (the staged leaves
                        fill the other positions in order) */
  uint64_t src_off;  /* element offsets */
  uint64_t dst_off;
  uint64_t aux_off;
  uint64_t count;    /* elements */
} bine_prim_t;

/* Fills up to `cap` primitives of rank `rank`'s plan; returns the number of
 * primitives (may exceed cap) or -status on error.  tmp_elems[3] receives the
 * workspace sizes (elements).  For reduce_scatter `count_or_root` is ignored and
 * rcounts is used; for reduce it is the root and `count` the element count. */
int64_t bine_plan(int algo, int nranks, int rank, size_t count, const int *rcounts, int root,
                  size_t esz, size_t segsize, int in_place, bine_prim_t *prims, int64_t cap,
                  uint64_t *tmp_elems);

/* The two-stream issue schedule the executor derives from a plan (inspection /
 * testing): one entry per primitive; entries with equal `op` form one unit of
 * work -- an exchange group on the comm stream (xchg = 1) or one local
 * primitive on the caller's stream.  `wait` = index of the op of the other
 * stream this op waits for (-1: none).  PIPELINE exchanges appear cut into
 * `chunk_bytes` pieces (0: uncut).  *c_join = 1 if the comm stream first waits
 * for the caller's prior work; *final_wait = op the caller's stream waits for
 * at the end (-1: none); workspace[4] = elements of TMP0, TMP1, TMP2 and the
 * relay staging buffer the schedule uses.
 * relay_min_bytes > 0 selects relay mode as bine_comm_set_relay does; `mode`
 * bit 0 = multi-tree mode (bine_comm_set_trees), bit 1 = flat allgather
 * (bine_comm_set_flat_ag), bit 2 = flat reduce-scatter (bine_comm_set_flat_rs),
 * bit 3 = the allgather cut with the flat reduce-scatter's chunks
 * (bine_comm_set_flat_ag(2)).  Returns the number of entries (may exceed cap)
 * or -status. */
typedef struct {
  int32_t op;
  int32_t xchg;
  int64_t wait;
  bine_prim_t prim;
} bine_sched_entry_t;

int64_t bine_plan_schedule(int algo, int nranks, int rank, size_t count, const int *rcounts, int root,
                           size_t esz, size_t segsize, int in_place, size_t chunk_bytes,
                           size_t relay_min_bytes, int mode, bine_sched_entry_t *out, int64_t cap,
                           int *c_join, int64_t *final_wait, uint64_t *workspace);

/* The host staging of that schedule (bine_allreduce_staged, no relay):
 * kind 0 = host->device pieces (op, lo, hi) in elements of the input buffer,
 * copied before op; kind 1 = device->host pieces (op, lo, hi) of RBUF,
 * copied after op; kind 2 = (op, h2d_wait): the newest op whose host->device
 * batch op waits for (-1 as UINT64_MAX: none).  `out` holds 3 (kinds 0, 1)
 * or 2 (kind 2) words per entry.  Returns the number of entries (may exceed
 * cap) or -status. */
/* The direct transport's fused-tree decisions (bine_comm_set_direct_tree)
 * for rank `rank`'s issue schedule, with the transport's shape rules at
 * sub-message slot `slot` and launch structure `merge` (BINE_DIRECT_MERGE):
 * host[i] = the exchange op whose launch evaluates tree op i (-1: not
 * fused), defer[i] = 1 when exchange op i's receives are pulled by the next
 * exchange (its tree deferred there).  Host only; `mode` as in
 * bine_plan_schedule.  Returns the number of ops (may exceed cap) or
 * -status. */
int64_t bine_plan_dm_trees(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                           int in_place, size_t chunk_bytes, int mode, size_t slot, int merge, int dtype, int op,
                           int32_t *host, int32_t *defer, int64_t cap);
int64_t bine_plan_stage(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                        size_t segsize, int in_place, size_t chunk_bytes, int mode, int kind, uint64_t *out,
                        int64_t cap);
/* Whether the direct transport issues rank `rank`'s call as k_dm_fused
 * launches (host only; the transport's slot `slot`, its fused trees on,
 * `mode` as in bine_plan_schedule, `small` = a single-stream call): the
 * number of launches, 0 when the call keeps its per-exchange launches, or
 * -status. */
int bine_plan_dm_fused(int algo, int nranks, int rank, size_t count, const int *rcounts, int root, size_t esz,
                       int in_place, size_t chunk_bytes, int mode, size_t slot, int dtype, int op, int small);
/* The same, with the launches' messages in the order their sequence numbers
 * are taken: 4 words each (launch, push, peer, bytes) into out (up to cap
 * messages; *nmsgs = how many there are).  Returns the launches or -status. */
int64_t bine_plan_dm_fused_msgs(int algo, int nranks, int rank, size_t count, const int *rcounts, int root,
                                size_t esz, int in_place, size_t chunk_bytes, int mode, size_t slot, int dtype, int op,
                                int small, uint64_t *out, int64_t cap, int64_t *nmsgs);

/* The direct transport's residency cut (host only): every launch's
 * workgroups -- `cw[0..n)` per copied message, *tw for a fused tree (NULL:
 * none) -- are scaled proportionally, each >= 1, to sum to at most `cap` =
 * CUs x (resident blocks per CU of the launched kernel - margin) / ranks
 * sharing the GPU (bine_dm_residency_cap), so that every waiting workgroup of
 * every co-located rank's current launch is resident at once, with a margin
 * for other waves, and no waiter can hold the slot its producer needs.
 * Returns 0 (unchanged: fits, or cap <= 0), 1 (scaled) or -1 (the parts alone
 * exceed cap; unchanged). */
int bine_dm_fit_residency(int *cw, int n, int *tw, int cap);
/* That cap on the current device (needs a GPU): kind 0 = k_dm_move, 1 =
 * k_dm_move_tree for (dtype, op, nl leaves), 2 = k_dm_fused for (dtype, op);
 * bine_dm_residency_cap(CUs, resident blocks per CU
 * (hipOccupancyMaxActiveBlocksPerMultiprocessor), margin, share) with the
 * margin of BINE_DIRECT_RESIDENCY_MARGIN (default 1).  -1: no such kernel; 0:
 * the device could not be queried. */
int bine_dm_launch_cap(int kind, int dtype, int op, int nl, int share);
/* The rule itself (host only): cus x max(1, per_cu - margin) / share -- the
 * margin is the blocks per CU left to waves other than the transport's
 * spinning ones; 0 when cus or per_cu <= 0. */
int bine_dm_residency_cap(int cus, int per_cu, int margin, int share);

#ifdef __cplusplus
}
#endif
#endif /* BINE_AMD_H */
