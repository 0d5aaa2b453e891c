// comm.h -- the gene-partial all-reduce over RCCL (xGMI), exported through the C-ABI.
//
// Replaces MergeGeneMetrics' CSV merge of cell-disjoint chunks (merge.py:74-191): every rank
// holds [rows][SCT_NP] int64 partial rows whose lanes are plain integer sums (counters and
// the exact fixed-point lanes of fixedpt.h), so ONE in-place ncclAllReduce(sum, int64) makes
// every rank's rows those of the union of the shards, bit for bit, in any rank order.
//
// The communicator helpers let a caller without torch.distributed build the ranks'
// communicators: one process driving several devices (ncclCommInitAll), or one process per
// device with an id exchanged out of band (ncclGetUniqueId / ncclCommInitRank).  A
// communicator from elsewhere (any ncclComm_t) is accepted as well.
#pragma once
#include <rccl/rccl.h>

#include "util.h"

#define NCCLCHK(expr)                                                                                 \
  do {                                                                                                \
    ncclResult_t _r = (expr);                                                                         \
    if (_r != ncclSuccess)                                                                            \
      return ::sct::fail(SCT_ENCCL, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__, \
                         __LINE__);                                                                   \
  } while (0)

extern "C" {

int sct_comm_unique_id(uint8_t* id, size_t bytes) {
  ::sct::last_error().clear();
  if (!id || bytes < sizeof(ncclUniqueId)) return ::sct::fail(SCT_EINVAL, "id buffer needs %zu bytes", sizeof(ncclUniqueId));
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return SCT_OK;
}

int sct_comm_init_rank(void** comm, int nranks, const uint8_t* id, size_t bytes, int rank, int device) {
  ::sct::last_error().clear();
  if (!comm || !id || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
    return ::sct::fail(SCT_EINVAL, "bad communicator arguments");
  HIPCHK(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  NCCLCHK(ncclCommInitRank(&c, nranks, u, rank));
  *comm = c;
  return SCT_OK;
}

int sct_comm_init_all(void** comms, int ndev, const int* devices) {
  ::sct::last_error().clear();
  if (!comms || !devices || ndev < 1) return ::sct::fail(SCT_EINVAL, "bad communicator arguments");
  NCCLCHK(ncclCommInitAll(reinterpret_cast<ncclComm_t*>(comms), ndev, devices));
  return SCT_OK;
}

int sct_comm_destroy(void* comm) {
  ::sct::last_error().clear();
  if (!comm) return SCT_OK;
  NCCLCHK(ncclCommDestroy(static_cast<ncclComm_t>(comm)));
  return SCT_OK;
}

int sct_comm_abort(void* comm) {
  ::sct::last_error().clear();
  if (!comm) return SCT_OK;
  NCCLCHK(ncclCommAbort(static_cast<ncclComm_t>(comm)));
  return SCT_OK;
}

int sct_allreduce_gene_partials(int64_t* partials, int64_t rows, void* comm, void* stream) {
  ::sct::last_error().clear();
  if (!comm) return ::sct::fail(SCT_EINVAL, "comm is NULL");
  if (rows < 0 || (rows > 0 && !partials)) return ::sct::fail(SCT_EINVAL, "bad partials");
  const size_t count = (size_t)rows * SCT_NP;
  NCCLCHK(ncclAllReduce(partials, partials, count, ncclInt64, ncclSum, static_cast<ncclComm_t>(comm),
                        (hipStream_t)stream));
  return SCT_OK;
}

}  // extern "C"
