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

// ---- the cell-bin exchange (SplitBam's bins between devices, bam.py:439-480) ----

int sct_exchange_counts(const int64_t* send_counts, int64_t* recv_counts, int32_t n_ranks, void* comm,
                        void* stream) {
  ::sct::last_error().clear();
  if (!comm || !send_counts || !recv_counts) return ::sct::fail(SCT_EINVAL, "NULL argument");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int nr = 0, me = 0;
  NCCLCHK(ncclCommCount(c, &nr));
  NCCLCHK(ncclCommUserRank(c, &me));
  if (nr != n_ranks) return ::sct::fail(SCT_EINVAL, "n_ranks %d but the communicator has %d ranks", n_ranks, nr);
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(recv_counts + me, send_counts + me, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  if (nr == 1) return SCT_OK;
  NCCLCHK(ncclGroupStart());
  for (int p = 0; p < nr; p++) {
    if (p == me) continue;
    NCCLCHK(ncclSend(send_counts + p, 1, ncclInt64, p, c, s));
    NCCLCHK(ncclRecv(recv_counts + p, 1, ncclInt64, p, c, s));
  }
  NCCLCHK(ncclGroupEnd());
  return SCT_OK;
}

int sct_exchange_records(const sct_records_t* binned, const int32_t* tiebreak, const int64_t* send_counts,
                         const int64_t* recv_counts, int32_t n_ranks, const sct_records_t* out,
                         int32_t* tiebreak_out, void* comm, void* stream) {
  ::sct::last_error().clear();
  if (!comm || !binned || !out || !send_counts || !recv_counts) return ::sct::fail(SCT_EINVAL, "NULL argument");
  if ((tiebreak == nullptr) != (tiebreak_out == nullptr))
    return ::sct::fail(SCT_EINVAL, "tiebreak and tiebreak_out: both or neither");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int nr = 0, me = 0;
  NCCLCHK(ncclCommCount(c, &nr));
  NCCLCHK(ncclCommUserRank(c, &me));
  if (nr != n_ranks) return ::sct::fail(SCT_EINVAL, "n_ranks %d but the communicator has %d ranks", n_ranks, nr);
  int64_t st = 0, rt = 0;
  for (int p = 0; p < nr; p++) {
    if (send_counts[p] < 0 || recv_counts[p] < 0) return ::sct::fail(SCT_EINVAL, "negative count for rank %d", p);
    st += send_counts[p];
    rt += recv_counts[p];
  }
  if (st != binned->n) return ::sct::fail(SCT_EINVAL, "send counts sum to %lld, binned.n is %lld", (long long)st,
                                          (long long)binned->n);
  if (rt != out->n) return ::sct::fail(SCT_EINVAL, "recv counts sum to %lld, out.n is %lld", (long long)rt,
                                       (long long)out->n);
  struct Col {
    const void* src;
    void* dst;
    size_t es;
  };
  const Col cols[15] = {{binned->cell, (void*)out->cell, 4},       {binned->umi, (void*)out->umi, 4},
                        {binned->gene, (void*)out->gene, 4},       {binned->ref, (void*)out->ref, 4},
                        {binned->pos, (void*)out->pos, 4},         {binned->gq_sum, (void*)out->gq_sum, 2},
                        {binned->gq_len, (void*)out->gq_len, 2},   {binned->gq_gt30, (void*)out->gq_gt30, 2},
                        {binned->bits, (void*)out->bits, 1},       {binned->xf, (void*)out->xf, 1},
                        {binned->cy_gt30, (void*)out->cy_gt30, 1}, {binned->cy_len, (void*)out->cy_len, 1},
                        {binned->uy_gt30, (void*)out->uy_gt30, 1}, {binned->uy_len, (void*)out->uy_len, 1},
                        {tiebreak, tiebreak_out, 4}};
  const int ncol = tiebreak ? 15 : 14;
  for (int k = 0; k < ncol; k++)
    if ((st && !cols[k].src) || (rt && !cols[k].dst)) return ::sct::fail(SCT_EINVAL, "NULL column %d", k);
  // offsets of the outgoing bins and of the incoming pieces
  std::vector<int64_t> so(nr + 1, 0), ro(nr + 1, 0);
  for (int p = 0; p < nr; p++) {
    so[p + 1] = so[p] + send_counts[p];
    ro[p + 1] = ro[p] + recv_counts[p];
  }
  if (send_counts[me] != recv_counts[me])
    return ::sct::fail(SCT_EINVAL, "own bin: %lld sent, %lld expected", (long long)send_counts[me],
                       (long long)recv_counts[me]);
  hipStream_t s = (hipStream_t)stream;
  for (int k = 0; k < ncol; k++)
    if (send_counts[me])
      HIPCHK(hipMemcpyAsync((uint8_t*)cols[k].dst + ro[me] * cols[k].es, (const uint8_t*)cols[k].src + so[me] * cols[k].es,
                            send_counts[me] * cols[k].es, hipMemcpyDeviceToDevice, s));
  if (nr == 1) return SCT_OK;
  NCCLCHK(ncclGroupStart());
  for (int k = 0; k < ncol; k++) {
    for (int p = 0; p < nr; p++) {
      if (p == me) continue;
      if (send_counts[p])
        NCCLCHK(ncclSend((const uint8_t*)cols[k].src + so[p] * cols[k].es, send_counts[p] * cols[k].es, ncclUint8, p, c, s));
      if (recv_counts[p])
        NCCLCHK(ncclRecv((uint8_t*)cols[k].dst + ro[p] * cols[k].es, recv_counts[p] * cols[k].es, ncclUint8, p, c, s));
    }
  }
  NCCLCHK(ncclGroupEnd());
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
