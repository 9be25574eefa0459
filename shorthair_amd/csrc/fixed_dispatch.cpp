// Dispatch to the compile-time-scheduled kernels generated for specific (k, m).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

#include "fixed_configs.h"  // from the generated-kernel directory (-I, see build.py)
#include "kernels.hpp"
#include "measure.hpp"

namespace sh {
namespace fixed {
#define SH_DECL(K, M)                                                    \
    hipError_t launch_k##K##_m##M##_enc(FixedArgs a, hipStream_t s);     \
    hipError_t launch_k##K##_m##M##_dec(FixedArgs a, hipStream_t s);
SH_FIXED_CONFIGS(SH_DECL)
#undef SH_DECL

// Measurement builds only (-DSH_MEASUREMENT_BUILD, tools/build_variant.sh): SH_HSACO_DIR=<dir>
// makes every compile-time kernel whose code object <dir>/<tag>.hsaco exists (tag =
// k<k>_m<m>_<enc|dec>, e.g. a tools/il_reorder.py layout of the same kernel) launch from that code
// object. The product library has neither the switch nor a module loader (measure.hpp).
hipError_t module_launch(const char *tag, const FixedArgs &a, unsigned blocks, unsigned threads, size_t lds,
                         hipStream_t s, bool *used) {
    *used = false;
#ifdef SH_MEASUREMENT_BUILD
    static const char *dir = SH_MEASURE_ENV("SH_HSACO_DIR");
    if (!dir) return hipSuccess;
    static std::mutex mu;
    static std::map<std::string, hipFunction_t> fns;
    hipFunction_t f = nullptr;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = fns.find(tag);
        if (it == fns.end()) {
            hipModule_t mod = nullptr;
            const std::string path = std::string(dir) + "/" + tag + ".hsaco";
            const std::string kname = std::string("kern_") + tag;
            const std::string sym = "_ZN2sh5fixed" + std::to_string(kname.size()) + kname + "ENS_9FixedArgsE";
            if (hipModuleLoad(&mod, path.c_str()) != hipSuccess || hipModuleGetFunction(&f, mod, sym.c_str()) != hipSuccess) {
                f = nullptr;
                (void)hipGetLastError();
            } else {
                std::fprintf(stderr, "libcauchy256: %s from %s\n", sym.c_str(), path.c_str());
            }
            it = fns.emplace(tag, f).first;
        }
        f = it->second;
    }
    if (!f) return hipSuccess;
    *used = true;
    FixedArgs arg = a;
    size_t sz = sizeof(arg);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &arg, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    return hipModuleLaunchKernel(f, blocks, 1, 1, threads, 1, 1, static_cast<unsigned>(lds), s, nullptr, cfg);
#else
    (void)tag, (void)a, (void)blocks, (void)threads, (void)lds, (void)s;
    return hipSuccess;
#endif
}

bool tag_is_module(const char *tag) {
#ifdef SH_MEASUREMENT_BUILD
    static const char *dir = SH_MEASURE_ENV("SH_HSACO_DIR");
    return dir && tag;
#else
    (void)tag;
    return false;
#endif
}
}  // namespace fixed

// A kernel compiled for (K, m) also codes k < K: the generator's column x is the same for every k
// (cauchy_256.cpp:423-481), and the steps past k read zeros. Those steps still run their XOR
// programs, so the kernel is used down to k = 0.6 K: at 6,000 groups of 1400 bytes the (224,32)
// kernel's full 224 steps took 0.585 ms against 0.674 for the tile kernel at (150,32), (200,56)
// 0.85 vs 1.25 at (150,56), (190,66) 0.98 vs 1.50 at (120,66) (profiles/r06/ab_runs.txt block 13).
int fixed_kernel_k(int k, int m, int B) {
    // the shifted last 16-byte chunk must stay inside its sub-block (B/8 >= 16; fixed_geometry)
    if (B % 8 != 0 || B / 8 < 16 || k < 1) return 0;
    int best = 0;
#define SH_FIT(K, M) \
    if (m == M && k <= K && (k == K || 10 * k >= 6 * K) && (best == 0 || K < best)) best = K;
    SH_FIXED_CONFIGS(SH_FIT)
#undef SH_FIT
    return best;
}

bool has_fixed(int k, int m, int B) { return fixed_kernel_k(k, m, B) > 0; }

hipError_t launch_fixed(int k, int m, FixedArgs a, bool dec, hipStream_t stream) {
    const int kk = fixed_kernel_k(k, m, a.geo.B);
    if (kk == 0) return hipErrorNotSupported;
    if (a.groups <= 0) return hipSuccess;
    a.k_rt = k;
#define SH_GO(K, M)                                                                         \
    if (kk == K && m == M)                                                                  \
        return dec ? fixed::launch_k##K##_m##M##_dec(a, stream) : fixed::launch_k##K##_m##M##_enc(a, stream);
    SH_FIXED_CONFIGS(SH_GO)
#undef SH_GO
    return hipErrorNotSupported;
}

}  // namespace sh
