// Dispatch to the compile-time-scheduled kernels generated for specific (k, m).
#include <hip/hip_runtime.h>

#include "fixed_configs.h"  // from the generated-kernel directory (-I, see build.py)
#include "kernels.hpp"

namespace sh {
namespace fixed {
#define SH_DECL(K, M)                                                    \
    hipError_t launch_k##K##_m##M##_enc(FixedArgs a, hipStream_t s);     \
    hipError_t launch_k##K##_m##M##_dec(FixedArgs a, hipStream_t s);
SH_FIXED_CONFIGS(SH_DECL)
#undef SH_DECL
}  // namespace fixed

bool has_fixed(int k, int m, int B) {
    // the shifted last 16-byte chunk must stay inside its sub-block (B/8 >= 16; fixed_geometry)
    if (B % 8 != 0 || B / 8 < 16) return false;
#define SH_HAS(K, M) if (k == K && m == M) return true;
    SH_FIXED_CONFIGS(SH_HAS)
#undef SH_HAS
    return false;
}

hipError_t launch_fixed(int k, int m, FixedArgs a, bool dec, hipStream_t stream) {
    if (!has_fixed(k, m, a.geo.B)) return hipErrorNotSupported;
    if (a.groups <= 0) return hipSuccess;
#define SH_GO(K, M)                                                                         \
    if (k == K && m == M)                                                                   \
        return dec ? fixed::launch_k##K##_m##M##_dec(a, stream) : fixed::launch_k##K##_m##M##_enc(a, stream);
    SH_FIXED_CONFIGS(SH_GO)
#undef SH_GO
    return hipErrorNotSupported;
}

}  // namespace sh
