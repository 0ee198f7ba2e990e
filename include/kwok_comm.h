/*
 * kwok_comm.h — the C5 cluster-aggregate collective without PyTorch.
 *
 * One process per GPU, each owning a node-block shard.  Once per reporting
 * interval every rank writes its engines' aggregates (kwk_aggregate: transitions per stage,
 * phase histograms, cluster usage; float64) into one device buffer and sums it across ranks
 * with a single RCCL all-reduce over xGMI — the only cross-GPU traffic of the path.  This
 * library is that collective for a host that is not Python: a Go controller links it beside
 * libkwok_engine and exchanges the 128-byte unique id out of band (the reference has no
 * collective at all: one kwok process per cluster talks to the apiserver; several kwok
 * processes split nodes by --manage-nodes-with-label-selector, controller.go:170-181).
 *
 * Ordering is by streams and events, no host synchronisation: kwk_comm_allreduce runs on the
 * communicator's own stream after all work queued so far on the given engines' streams, and the
 * engines' later work waits for it (the next interval rewrites the buffer).
 */
#ifndef KWOK_COMM_H
#define KWOK_COMM_H

#include <stdint.h>

#include "kwok_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kwk_comm kwk_comm;
#define KWK_COMM_ID_BYTES 128  /* ncclUniqueId */

/* message of the last failing call on c (per communicator); c = NULL: the calling thread's */
const char* kwk_comm_last_error(const kwk_comm* c);
/* rank 0 creates the id and shares it with the other ranks (out of band) */
kwk_status kwk_comm_unique_id(uint8_t id[KWK_COMM_ID_BYTES]);
/* collective over all ranks (ncclCommInitRank): blocks until every rank has joined */
kwk_status kwk_comm_init(const uint8_t id[KWK_COMM_ID_BYTES], int32_t rank, int32_t world, int32_t device,
                         kwk_comm** out);
kwk_status kwk_comm_destroy(kwk_comm* c);
/* a device buffer of n float64 owned by the communicator (reallocated when n grows): the target
 * of kwk_aggregate(eng, ..., out = *dev + offset, ...) for each engine.  Growing it frees the
 * previous buffer: every pointer an earlier call returned is invalid from then on (size the
 * buffer once, for all the reports that share the communicator, before handing pointers out) */
kwk_status kwk_comm_buffer(kwk_comm* c, uint64_t n, double** dev);
/* in-place sum of the first n doubles of the buffer across all ranks, ordered after the work
 * queued on `engines` and before their later work (enqueue only) */
kwk_status kwk_comm_allreduce(kwk_comm* c, uint64_t n, kwk_engine* const* engines, uint32_t n_engines);
/* copies the first n doubles of the buffer to host memory after the last all-reduce (synchronises) */
kwk_status kwk_comm_read(kwk_comm* c, double* host_out, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif /* KWOK_COMM_H */
