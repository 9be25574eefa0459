// Dispatch to the compile-time-scheduled kernels generated for specific (k, m).
#include <hip/hip_runtime.h>

#include "fixed_configs.h"  // from the generated-kernel directory (-I, see build.py)
#include "kernels.hpp"

namespace sh {
namespace fixed {
#define SH_DECL(K, M) hipError_t launch_k##K##_m##M(FixedArgs a, bool dec, hipStream_t s);
SH_FIXED_CONFIGS(SH_DECL)
#undef SH_DECL
}  // namespace fixed

bool has_fixed(int k, int m, int B) {
    if (B % 8 != 0 || B / 8 < 4) return false;
#define SH_HAS(K, M) if (k == K && m == M) return true;
    SH_FIXED_CONFIGS(SH_HAS)
#undef SH_HAS
    return false;
}

hipError_t launch_fixed(int k, int m, FixedArgs a, bool dec, hipStream_t stream) {
    if (!has_fixed(k, m, a.geo.B)) return hipErrorNotSupported;
    if (a.groups <= 0) return hipSuccess;
#define SH_GO(K, M) if (k == K && m == M) return fixed::launch_k##K##_m##M(a, dec, stream);
    SH_FIXED_CONFIGS(SH_GO)
#undef SH_GO
    return hipErrorNotSupported;
}

}  // namespace sh
