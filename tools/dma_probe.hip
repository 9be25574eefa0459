// Probe: does buffer_load_dwordx4 ... lds (gfx950 LDS-DMA) handle byte-misaligned sources, and what
// does it write for partially / fully out-of-range chunks? Prints a verdict per case.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_t;

// Each lane DMAs 16 bytes from in[base + 16*lane] (base arbitrary) into LDS, then copies LDS out.
__global__ __launch_bounds__(64) void k_dma16(const uint8_t *in, uint32_t nrec, uint32_t base, uint8_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)nrec, 0x00020000);
    for (int i = threadIdx.x; i < 1024 / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = 0xA5A5A5A5u;
    __syncthreads();
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t *)lds, 16, base + 16 * threadIdx.x, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

__global__ __launch_bounds__(64) void k_dma4(const uint8_t *in, uint32_t nrec, uint32_t base, uint8_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(in), (short)0, (int)nrec, 0x00020000);
    for (int i = threadIdx.x; i < 256 / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = 0xA5A5A5A5u;
    __syncthreads();
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t *)lds, 4, base + 4 * threadIdx.x, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}

static int check(const char *name, const uint8_t *host_in, uint32_t nrec, uint32_t base, const uint8_t *got, int width) {
    int bad = 0, oob_zero = 0, oob_other = 0;
    for (int i = 0; i < 64 * width; ++i) {
        uint32_t off = base + i;
        if (off < nrec) {
            if (got[i] != host_in[off]) ++bad;
        } else {
            if (got[i] == 0) ++oob_zero; else ++oob_other;
        }
    }
    // bytes in range but inside a dword that straddles nrec
    int straddle_bad = 0;
    for (int i = 0; i < 64 * width; ++i) {
        uint32_t off = base + i;
        if (off < nrec && got[i] != host_in[off]) { ++straddle_bad; if (straddle_bad < 4) printf("    mismatch at lane-byte %d (off %u): got %02x want %02x\n", i, off, got[i], host_in[off]); }
    }
    printf("%-34s base=%-6u nrec=%-6u in-range mismatches=%d oob_zero=%d oob_other=%d\n", name, base, nrec, bad, oob_zero, oob_other);
    return bad;
}

int main() {
    const int N = 1 << 16;
    uint8_t *h = (uint8_t *)malloc(N);
    for (int i = 0; i < N; ++i) h[i] = (uint8_t)(i * 131 + 7 + (i >> 8));
    uint8_t *d_in, *d_out;
    CK(hipMalloc(&d_in, N));
    CK(hipMalloc(&d_out, 1024));
    CK(hipMemcpy(d_in, h, N, hipMemcpyHostToDevice));
    uint8_t got[1024];
    int fails = 0;
    uint32_t bases[] = {0, 1, 2, 3, 175, 350, 1227, 4097};
    for (uint32_t b : bases) {
        hipLaunchKernelGGL(k_dma16, dim3(1), dim3(64), 1024, 0, d_in, (uint32_t)N, b, d_out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got, d_out, 1024, hipMemcpyDeviceToHost));
        char nm[64]; snprintf(nm, sizeof nm, "dwordx4 misalign %u", b & 15);
        fails += check(nm, h, N, b, got, 16) != 0;
        hipLaunchKernelGGL(k_dma4, dim3(1), dim3(64), 256, 0, d_in, (uint32_t)N, b, d_out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got, d_out, 256, hipMemcpyDeviceToHost));
        snprintf(nm, sizeof nm, "dword misalign %u", b & 3);
        fails += check(nm, h, N, b, got, 4) != 0;
    }
    // out-of-range: nrec cuts the wave's span at various points (inside a dword, at a dword edge)
    uint32_t cuts[] = {1000, 1001, 1003, 1005, 1012};
    for (uint32_t c : cuts) {
        for (uint32_t b : {0u, 1u, 3u}) {
            hipLaunchKernelGGL(k_dma16, dim3(1), dim3(64), 1024, 0, d_in, c, b, d_out);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got, d_out, 1024, hipMemcpyDeviceToHost));
            check("dwordx4 OOB cut", h, c, b, got, 16);
        }
    }
    printf(fails ? "VERDICT: misaligned LDS-DMA NOT exact\n" : "VERDICT: misaligned LDS-DMA exact\n");
    return 0;
}
