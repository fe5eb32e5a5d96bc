// Instantiations of the temporal-blocking kernel (jacobi5tb.hpp) for K = 1, 2, 3, 4, 5, 6, 7.
#include "jacobi5tb.hpp"

namespace gmt {
namespace tb {
template int dispatch_k<1>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<2>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<3>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<4>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<5>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<6>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<7>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
}  // namespace tb
}  // namespace gmt
