// Host-backend stub of gmt/ccl.h: there are no device collectives without a
// GPU, so every call reports GMT_CCL_UNAVAILABLE and the transports fall back
// to MPI (gmt::comm::resolve never picks rccl when gmt_ccl_available() == 0).
#include "gmt/ccl.h"

extern "C" {

int gmt_ccl_available(void) { return 0; }
const char* gmt_ccl_error_string(int) { return "RCCL not available in the host backend"; }
int gmt_ccl_version(int* v) {
  *v = 0;
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_get_unique_id(gmt_ccl_id*) { return GMT_CCL_UNAVAILABLE; }
int gmt_ccl_comm_init(gmt_ccl_comm_t* c, int, const gmt_ccl_id*, int) {
  *c = nullptr;
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_comm_destroy(gmt_ccl_comm_t) { return 0; }
int gmt_ccl_group_start(void) { return GMT_CCL_UNAVAILABLE; }
int gmt_ccl_group_end(void) { return GMT_CCL_UNAVAILABLE; }
int gmt_ccl_send(const void*, size_t, int, gmt_ccl_comm_t, gmt_stream_t) {
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_recv(void*, size_t, int, gmt_ccl_comm_t, gmt_stream_t) { return GMT_CCL_UNAVAILABLE; }
int gmt_ccl_allreduce_sum_f64(const double*, double*, size_t, gmt_ccl_comm_t, gmt_stream_t) {
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_allreduce_max_f64(const double*, double*, size_t, gmt_ccl_comm_t, gmt_stream_t) {
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_allgather(const void*, void*, size_t, gmt_ccl_comm_t, gmt_stream_t) {
  return GMT_CCL_UNAVAILABLE;
}
int gmt_ccl_broadcast(void*, size_t, int, gmt_ccl_comm_t, gmt_stream_t) {
  return GMT_CCL_UNAVAILABLE;
}

}  // extern "C"
