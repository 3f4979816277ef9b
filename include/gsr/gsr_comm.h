/*
 * gsr_comm.h -- C ABI of the multi-GPU transport: RCCL over xGMI for the three
 * data-path exchanges of one sharded step (gsr.h "Multi-GPU"), in the same libgsr_hip.so.
 * The reference has no distributed code at all (SURVEY §2 ★E); this is the boundary a C++
 * training loop (src/utils/train_utils.cpp:97-146) reaches the collectives through, so that its
 * host code stays C++ and calls HIP / RCCL only through libgsr_hip.so.
 *
 *   gsr_comm_all_to_all     splat blocks shard -> band, and the 2D-gradient rows back: ONE group
 *                           of ncclSend / ncclRecv pairs (xGMI is a full mesh of point-to-point
 *                           links, so each pair moves over its own link -- no ring)
 *   gsr_comm_all_gather     the band images (+ each rank's overflow status words)
 *   gsr_comm_all_reduce_i64 setup only: the summed row histogram, the largest splat count
 *
 * Conventions as gsr.h: device pointers, one hipStream_t, 0 = ok / < 0 = error with the message
 * in gsr_last_error of gsr.h.  Every call is stream-ordered and may be recorded into a hipGraph
 * (stream capture).  One communicator per rank; ranks are processes, one GPU each.
 */
#ifndef GSR_GSR_COMM_H
#define GSR_GSR_COMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_COMM_ID_BYTES 128 /* = NCCL_UNIQUE_ID_BYTES */

typedef struct gsr_comm gsr_comm;

/* Rank 0 creates the id; the caller hands it to every rank (a store, torch.distributed, MPI). */
int gsr_comm_unique_id(uint8_t id[GSR_COMM_ID_BYTES]);
/* Collective over `world` processes (blocks until all ranks have called it). */
int gsr_comm_init(gsr_comm** comm, const uint8_t id[GSR_COMM_ID_BYTES], int32_t world, int32_t rank);
int gsr_comm_destroy(gsr_comm* comm);
/* The communicator's size and this rank, as RCCL reports them (ncclCommCount / ncclCommUserRank):
 * what a benchmark line quotes as its GPU count. */
int gsr_comm_size(gsr_comm* comm, int32_t* world, int32_t* rank);

/* Block b of send (block_bytes each) -> rank b; block s of recv <- rank s. */
int gsr_comm_all_to_all(gsr_comm* comm, const void* send, void* recv, size_t block_bytes, void* stream);
/* `bytes` from every rank into recv, rank-major. */
int gsr_comm_all_gather(gsr_comm* comm, const void* send, void* recv, size_t bytes, void* stream);
/* In place; op 0 = sum, 1 = max. */
int gsr_comm_all_reduce_i64(gsr_comm* comm, int64_t* buf, size_t n, int32_t op, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_GSR_COMM_H */
