/*
 * libbine_amd.h -- the drop-in C ABI: the function set of the reference's
 * include/libbine.h (HLC-Lab/pico, include/libbine.h:12-78), exported by
 * pico_amd/lib/libbine.so with identical names and MPI-typed signatures, so
 * that pico_core (and anything else linking -lbine) runs unchanged on MI355X.
 *
 *   reference                                 here
 *   ---------------------------------------   -----------------------------------------
 *   size_t bine_allreduce_segsize   :28       same global, read by the segmented variant
 *   allreduce_*                    :30-37     GPU path (bine_allreduce, RCCL + HIP kernels)
 *   reduce_bine_lat / _bdw         :64-65     GPU path (bine_reduce)
 *   reduce_scatter_*               :69-77     GPU path (bine_reduce_scatter)
 *   allgather_*                    :39-50     GPU path (bine_allgather)
 *   bcast_*                        :54-60     GPU path (bine_bcast)
 *   alltoall_bine, gather_bine,    :52,63,78  GPU path (bine_alltoall / _gather /
 *   scatter_bine                              _scatter); data movement, run on bytes
 *
 * Buffers may be host or device memory (hipPointerGetAttributes decides):
 * device buffers are used in place; host buffers (pico_core's default
 * allocators, pico_core_allreduce_utils.c:13-25) are staged through cached
 * device buffers (H2D, device collective, D2H).  MPI_IN_PLACE is honoured.
 * Every call is complete on return (the reference's blocking semantics).
 * Rank -> GPU: local rank within MPI_COMM_TYPE_SHARED modulo the visible device
 * count (override: BINE_DEVICE).  One RCCL communicator per MPI communicator,
 * created on first use (ncclUniqueId broadcast over MPI) and cached as an MPI
 * attribute; all are released from an MPI_COMM_SELF delete callback at
 * MPI_Finalize.  Errors come back as MPI error classes, never exit().
 */
#ifndef LIBBINE_AMD_H
#define LIBBINE_AMD_H

#include <mpi.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BINE_ALLREDUCE_ARGS const void *sbuf, void *rbuf, size_t count, MPI_Datatype dtype, MPI_Op op, MPI_Comm comm
#define BINE_ALLGATHER_ARGS const void *sbuf, size_t scount, MPI_Datatype sdtype, void *rbuf, size_t rcount, \
                            MPI_Datatype rdtype, MPI_Comm comm
#define BINE_BCAST_ARGS void *buf, size_t count, MPI_Datatype dtype, int root, MPI_Comm comm
#define BINE_GATHER_ARGS const void *sbuf, size_t scount, MPI_Datatype sdtype, void *rbuf, size_t rcount, \
                         MPI_Datatype rdtype, int root, MPI_Comm comm
#define BINE_REDUCE_ARGS const void *sbuf, void *rbuf, size_t count, MPI_Datatype dtype, MPI_Op op, int root, \
                         MPI_Comm comm
#define BINE_REDUCE_SCATTER_ARGS const void *sbuf, void *rbuf, const int rcounts[], MPI_Datatype dtype, \
                                 MPI_Op op, MPI_Comm comm

extern size_t bine_allreduce_segsize;

/* reduce family: the MI355X path */
int allreduce_recursivedoubling(BINE_ALLREDUCE_ARGS);
int allreduce_ring(BINE_ALLREDUCE_ARGS);
int allreduce_rabenseifner(BINE_ALLREDUCE_ARGS);
int allreduce_bine_lat(BINE_ALLREDUCE_ARGS);
int allreduce_bine_bdw_static(BINE_ALLREDUCE_ARGS);
int allreduce_bine_bdw_remap(BINE_ALLREDUCE_ARGS);
int allreduce_bine_bdw_remap_segmented(BINE_ALLREDUCE_ARGS);
int allreduce_bine_block_by_block_any_even(BINE_ALLREDUCE_ARGS);

int reduce_bine_lat(BINE_REDUCE_ARGS);
int reduce_bine_bdw(BINE_REDUCE_ARGS);

int reduce_scatter_recursivehalving(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_recursive_distance_doubling(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_ring(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_butterfly(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_bine_static(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_bine_send_remap(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_bine_permute_remap(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_bine_block_by_block(BINE_REDUCE_SCATTER_ARGS);
int reduce_scatter_bine_block_by_block_any_even(BINE_REDUCE_SCATTER_ARGS);

/* data movement: allgather, alltoall, bcast, gather, scatter */
int allgather_k_bruck(BINE_ALLGATHER_ARGS);
int allgather_recursivedoubling(BINE_ALLGATHER_ARGS);
int allgather_ring(BINE_ALLGATHER_ARGS);
int allgather_sparbit(BINE_ALLGATHER_ARGS);
int allgather_bine_block_by_block(BINE_ALLGATHER_ARGS);
int allgather_bine_block_by_block_any_even(BINE_ALLGATHER_ARGS);
int allgather_bine_permute_static(BINE_ALLGATHER_ARGS);
int allgather_bine_send_static(BINE_ALLGATHER_ARGS);
int allgather_bine_permute_remap(BINE_ALLGATHER_ARGS);
int allgather_bine_send_remap(BINE_ALLGATHER_ARGS);
int allgather_bine_2_blocks(BINE_ALLGATHER_ARGS);
int allgather_bine_2_blocks_dtype(BINE_ALLGATHER_ARGS);
int alltoall_bine(BINE_ALLGATHER_ARGS);
int bcast_scatter_allgather(BINE_BCAST_ARGS);
int bcast_bine_lat(BINE_BCAST_ARGS);
int bcast_bine_lat_reversed(BINE_BCAST_ARGS);
int bcast_bine_lat_new(BINE_BCAST_ARGS);
int bcast_bine_lat_i_new(BINE_BCAST_ARGS);
int bcast_bine_bdw_static(BINE_BCAST_ARGS);
int bcast_bine_bdw_remap(BINE_BCAST_ARGS);
int gather_bine(BINE_GATHER_ARGS);
int scatter_bine(BINE_GATHER_ARGS);

#ifdef __cplusplus
}
#endif
#endif /* LIBBINE_AMD_H */
