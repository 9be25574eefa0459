#!/usr/bin/env python3
"""Generate tools/issue_probe.hip: VALU issue-rate probe for bitop3 streams (measurement only).

Question it answers: at the occupancy of the compile-time kernels (4 waves/SIMD), how many cycles
per SIMD does a stream of independent v_bitop3_b32 cost, and how much of that is instruction
supply (fetch bandwidth, straight-line code larger than the instruction cache, several distinct
code streams per CU) rather than the VALU itself?

Variants (one kernel each; every wave runs the same number of VALU instructions):
  loop_b3      64 bitop3 (8 B) per iteration of a tight loop            -> small code, 8-B instrs
  loop_x2      64 v_xor_b32 (4 B) per iteration                          -> small code, 4-B instrs
  loop_b3ds    64 bitop3 + 8 ds_read_b32 per iteration (the step mix)
  line_b3_1    LINE bitop3 straight-line, every wave the same code       -> big code, 1 stream
  line_b3_4    four straight-line copies, wave w runs copy w % 4         -> big code, 4 streams/WG
  line_x2_1    LINE v_xor_b32 straight-line, one stream
Usage: python tools/issue_probe_gen.py && hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools/issue_probe
"""
import os

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
LINE = 8192  # straight-line instructions per copy (64 KB of bitop3)


def b3(i, salt=0):
    # acc v[i%64] ^= t[a] ^ t[b]; tables v[64..95]; sources in three different banks (reg % 4)
    d = i % 64
    a = 64 + ((i * 5 + salt) % 16) * 2          # even -> banks 0/2
    b = 65 + ((i * 3 + 7 * salt) % 16) * 2      # odd  -> banks 1/3
    if (a % 4) == (d % 4):
        a = 64 + ((a - 64 + 2) % 32)
    if (b % 4) == (d % 4) or (b % 4) == (a % 4):
        b = 65 + ((b - 65 + 2) % 32)
    return f"v_bitop3_b32 v{d}, v{d}, v{a}, v{b} bitop3:0x96"


def x2(i, salt=0):
    d = i % 64
    a = 64 + ((i * 5 + salt) % 32)
    if (a % 4) == (d % 4):
        a = 64 + ((a - 64 + 1) % 32)
    return f"v_xor_b32 v{d}, v{a}, v{d}"


def asm_block(lines):
    return "\n".join(f'        "{l}\\n"' for l in lines)


CLOB = ", ".join(f'"v{i}"' for i in range(105))


def kernel(name, body, loop):
    """body: list of asm lines; loop: iterations variable name or None."""
    out = [f"__global__ __launch_bounds__(256) void k_{name}(unsigned long long *st, int iters) {{",
           "    __shared__ unsigned int lds_buf[1024];",
           "    lds_buf[threadIdx.x] = threadIdx.x;",
           "    __syncthreads();",
           "    unsigned long long t0 = __builtin_amdgcn_s_memtime();",
           "    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();",
           '    asm volatile("" ::: "memory");',
           "    for (int it = 0; it < iters; ++it) {",
           "        asm volatile(",
           asm_block(body),
           f"        ::: {CLOB});",
           "    }",
           '    asm volatile("" ::: "memory");',
           "    unsigned long long t1 = __builtin_amdgcn_s_memtime();",
           "    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();",
           "    if ((threadIdx.x & 63) == 0) {",
           "        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);",
           "        st[4 * w + 0] = t0; st[4 * w + 1] = t1 + lds_buf[(threadIdx.x + 1) & 255]; st[4 * w + 2] = r0; st[4 * w + 3] = r1;",
           "    }",
           "}"]
    return "\n".join(out)


def kernel_4way(name, bodies):
    out = [f"__global__ __launch_bounds__(256) void k_{name}(unsigned long long *st, int iters) {{",
           "    const int sel = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 3;",
           "    unsigned long long t0 = __builtin_amdgcn_s_memtime();",
           "    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();",
           '    asm volatile("" ::: "memory");',
           "    for (int it = 0; it < iters; ++it) {"]
    for s, body in enumerate(bodies):
        kw = "if" if s == 0 else "else if"
        out += [f"        {kw} (sel == {s}) asm volatile(", asm_block(body), f"        ::: {CLOB});"]
    out += ["    }",
            '    asm volatile("" ::: "memory");',
            "    unsigned long long t1 = __builtin_amdgcn_s_memtime();",
            "    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();",
            "    if ((threadIdx.x & 63) == 0) {",
            "        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);",
            "        st[4 * w + 0] = t0; st[4 * w + 1] = t1; st[4 * w + 2] = r0; st[4 * w + 3] = r1;",
            "    }",
            "}"]
    return "\n".join(out)


def main():
    ks = []
    ks.append(("loop_b3", kernel("loop_b3", [b3(i) for i in range(64)], True), 64, LINE // 64))
    ks.append(("loop_x2", kernel("loop_x2", [x2(i) for i in range(64)], True), 64, LINE // 64))
    mix = ["v_mov_b32 v104, 0"]
    for i in range(64):
        mix.append(b3(i))
        if i % 8 == 0:
            mix.append(f"ds_read_b32 v{96 + i // 8}, v104 offset:{(i // 8) * 512}")
    mix.append("s_waitcnt lgkmcnt(0)")
    ks.append(("loop_b3ds", kernel("loop_b3ds", mix, True), 64, LINE // 64))
    ks.append(("line_b3_1", kernel("line_b3_1", [b3(i, i // 64) for i in range(LINE)], True), LINE, 1))
    ks.append(("line_b3_4", kernel_4way("line_b3_4", [[b3(i, i // 64 + 17 * s) for i in range(LINE)] for s in range(4)]), LINE, 1))
    ks.append(("line_x2_1", kernel("line_x2_1", [x2(i, i // 64) for i in range(LINE)], True), LINE, 1))
    src = ["// GENERATED by tools/issue_probe_gen.py -- measurement only, not part of the product.",
           "#include <hip/hip_runtime.h>", "#include <stdio.h>", "#include <stdlib.h>", "#include <string.h>", "",
           "#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf(\"%s\\n\", hipGetErrorString(e_)); exit(1); } } while (0)", ""]
    for _, k, _, _ in ks:
        src.append(k)
        src.append("")
    src.append("typedef void (*kfn)(unsigned long long *, int);")
    src.append("struct V { const char *name; kfn f; int per_iter; int mult; };")
    src.append("static V vars[] = {" + ", ".join(f'{{"{n}", k_{n}, {p}, {m}}}' for n, _, p, m in ks) + "};")
    src.append(r'''
// issue_probe VARIANT BLOCKS_PER_CU REPS   (REPS x LINE instructions per wave)
int main(int argc, char **argv) {
    const char *which = argc > 1 ? argv[1] : "all";
    const int bpc = argc > 2 ? atoi(argv[2]) : 4;
    const int reps = argc > 3 ? atoi(argv[3]) : 64;
    const int ncu = 256, nb = ncu * bpc, nw = nb * 4;
    unsigned long long *st;
    CK(hipMalloc(&st, sizeof(unsigned long long) * 4 * nw));
    unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * 4 * nw);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &v : vars) {
        if (strcmp(which, "all") && strcmp(which, v.name)) continue;
        const int iters = reps * v.mult;
        for (int pass = 0; pass < 3; ++pass) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.f, dim3(nb), dim3(256), 0, 0, st, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(h, st, sizeof(unsigned long long) * 4 * nw, hipMemcpyDeviceToHost));
            double cyc = 0, rt = 0;
            for (int w = 0; w < nw; ++w) { cyc += h[4 * w + 1] - h[4 * w]; rt += h[4 * w + 3] - h[4 * w + 2]; }
            cyc /= nw; rt /= nw;
            const double ghz = cyc / (rt * 10.0);  // memrealtime = 100 MHz
            const double instr = (double)iters * v.per_iter;            // per wave
            const double waves_per_simd = bpc;                          // 4 waves per block, 1 per SIMD
            // cycles per instruction per SIMD from the wave's own stamps (all waves of a SIMD run together)
            const double cpi = cyc / (instr * waves_per_simd);
            const double wall_cpi = (ms * 1e-3) * ghz * 1e9 / (instr * waves_per_simd);
            if (pass == 2)
                printf("%-10s waves/SIMD=%d  %.3f ms  clock %.2f GHz  cycles/instr/SIMD: stamps %.2f wall %.2f\n",
                       v.name, bpc, ms, ghz, cpi, wall_cpi);
        }
    }
    return 0;
}
''')
    with open(os.path.join(ROOT, "tools", "issue_probe.hip"), "w") as f:
        f.write("\n".join(src) + "\n")


if __name__ == "__main__":
    main()
