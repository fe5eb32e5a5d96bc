/*
 * gmt/ccl.h — collective / point-to-point device communication C ABI.
 *
 * HIP build: RCCL over xGMI (csrc/runtime/ccl_rccl.cpp).  Host build: the
 * same semantics emulated over Unix-domain sockets between the processes of
 * one node (csrc/host/ccl_host.cpp): gmt_ccl_available() == 0 (automatic
 * transport selection never picks it) and gmt_ccl_emulated() == 1 (an
 * explicit "rccl" request runs on it).
 *
 * The reference passes device pointers straight to GPU-aware MPI
 * (MPI_Isend/Irecv: mpi_stencil2d_gt.cc:186-225, MPI_Allreduce :615,
 * MPI_Allgather: mpi_daxpy_nvtx.cc:285-288).  On an MI355X node the data
 * plane for those calls is RCCL: stream-ordered, xGMI peer links, no host
 * round trip.  MPI stays the control plane (it broadcasts the unique id).
 */
#ifndef GMT_CCL_H
#define GMT_CCL_H

#include <stddef.h>

#include "gmt/rt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GMT_CCL_UNAVAILABLE 9001
/* gmt_ccl_comm_init gave up: not every rank joined within
 * GMT_CCL_INIT_TIMEOUT seconds (default 300 with RCCL, 120 emulated) */
#define GMT_CCL_TIMEOUT 9004

typedef struct gmt_ccl_comm_s* gmt_ccl_comm_t;
typedef struct gmt_ccl_id {
  char internal[128]; /* ncclUniqueId */
} gmt_ccl_id;

int gmt_ccl_available(void);
int gmt_ccl_emulated(void);
const char* gmt_ccl_error_string(int err);
int gmt_ccl_version(int* v);
int gmt_ccl_get_unique_id(gmt_ccl_id* id);
int gmt_ccl_comm_init(gmt_ccl_comm_t* comm, int nranks, const gmt_ccl_id* id, int rank);
int gmt_ccl_comm_destroy(gmt_ccl_comm_t comm);
int gmt_ccl_group_start(void);
int gmt_ccl_group_end(void);
int gmt_ccl_send(const void* buf, size_t bytes, int peer, gmt_ccl_comm_t comm, gmt_stream_t s);
int gmt_ccl_recv(void* buf, size_t bytes, int peer, gmt_ccl_comm_t comm, gmt_stream_t s);
/* in place when send == recv */
int gmt_ccl_allreduce_sum_f64(const double* send, double* recv, size_t count,
                              gmt_ccl_comm_t comm, gmt_stream_t s);
int gmt_ccl_allreduce_max_f64(const double* send, double* recv, size_t count,
                              gmt_ccl_comm_t comm, gmt_stream_t s);
/* recv holds nranks * bytes_per_rank; in place when send == recv + rank*bytes */
int gmt_ccl_allgather(const void* send, void* recv, size_t bytes_per_rank,
                      gmt_ccl_comm_t comm, gmt_stream_t s);
int gmt_ccl_broadcast(void* buf, size_t bytes, int root, gmt_ccl_comm_t comm, gmt_stream_t s);

#ifdef __cplusplus
}
#endif
#endif /* GMT_CCL_H */
