// Instantiations of the temporal-blocking kernel (jacobi5tb.hpp) for K = 14, 16.
#include "jacobi5tb.hpp"

namespace gmt {
namespace tb {
template int dispatch_k<14>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
template int dispatch_k<16>(const gmt_tb_opts&, bool, int, const int64_t*, const int64_t*, int, const double*,
                               double*, int64_t, int64_t, hipStream_t, int64_t*);
}  // namespace tb
}  // namespace gmt
