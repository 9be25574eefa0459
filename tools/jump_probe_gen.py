#!/usr/bin/env python3
"""Generate tools/jump_probe.hip: cost of reaching a runtime-selected code snippet (measurement only).

The runtime-coefficient kernels (csrc/tile_snip.hip, decode stage B) apply M(c) for a
wave-uniform runtime c by calling one of 256 compile-time snippets (8 v_bitop3_b32 each). This
probe times, at 1/2/4/8 waves per SIMD, 8 products per loop iteration in these forms:
  inline    the 8 bitop3 of each product inline (no jump): the floor
  call72    s_swappc into a 72-byte-stride snippet table, s_setpc back (the product's form)
  call128   the same with each snippet 128-byte aligned (one fetch window per snippet)
  direct    s_branch to a fixed snippet and s_branch back (direct, PC-relative jumps)
  setpc1    s_setpc into the snippet, which ends with s_branch to a fixed return label (one
            indirect jump per product instead of two)
Usage: python tools/jump_probe_gen.py && hipcc --offload-arch=gfx950 -O3 tools/jump_probe.hip -o tools/jump_probe
"""
import os

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
ACC, T0, T1 = 32, 96, 112


def gmul2(v):
    v <<= 1
    return v ^ 0x187 if v & 0x100 else v


def snippet(c, ret):
    out, v = [], c
    for b in range(8):
        out.append(f"v_bitop3_b32 v{ACC + b}, v{ACC + b}, v{T0 + (v & 15)}, v{T1 + (v >> 4)} bitop3:0x96")
        v = gmul2(v)
    return out + ret


def table(label, align, ret):
    lines = [f".p2align {align}", f"{label}:"]
    for c in range(256):
        lines.append(f".p2align {align}")
        lines += snippet(c, ret)
    return lines


COEF = [0x53, 0xCA, 0x1F, 0x8E, 0x35, 0xB2, 0x67, 0xD9]


def body(mode):
    L = []
    if mode == "noidx":  # absolute registers, no VGPR-index mode
        for j, c in enumerate(COEF):
            v = c
            for b in range(8):
                L.append(f"v_bitop3_b32 v{ACC + 8 * j + b}, v{ACC + 8 * j + b}, v{T0 + (v & 15)}, v{T1 + (v >> 4)} bitop3:0x96")
                v = gmul2(v)
    elif mode == "idx0":  # VGPR-index mode on, M0 never changed inside
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            L += snippet(c, [])
        L.append("s_set_gpr_idx_off")
    elif mode == "idxnop":  # as inline, with s_nop 1 after each index change
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
                L.append("s_nop 1")
            L += snippet(c, [])
        L.append("s_set_gpr_idx_off")
    elif mode == "inline":
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L += snippet(c, [])
        L.append("s_set_gpr_idx_off")
    elif mode in ("call72", "call128"):
        stride = 72 if mode == "call72" else 128
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L.append(f"s_add_u32 s42, s44, {stride * c}")
            L.append("s_addc_u32 s43, s45, 0")
            L.append("s_swappc_b64 s[40:41], s[42:43]")
        L.append("s_set_gpr_idx_off")
    elif mode == "v2":  # stage B v2's form: snippet address from a coefficient word by SALU
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j in range(8):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            w = "s50" if j < 4 else "s51"
            L += [f"s_bfe_u32 s42, {w}, {0x80000 + 8 * (j % 4)}", "s_lshl3_add_u32 s42, s42, s42",
                  "s_lshl3_add_u32 s42, s42, s44", "s_mov_b32 s43, s45", "s_swappc_b64 s[40:41], s[42:43]"]
        L.append("s_set_gpr_idx_off")
    elif mode == "rl":  # snippet address low dwords from a VGPR (lane j) by v_readlane, before idx mode
        # (in VGPR-index mode SRC0 of v_readlane would be M0-relative)
        L += [f"v_readlane_b32 s{52 + j}, v20, {j}" for j in range(8)]
        L.append("s_mov_b32 s43, s45")
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j in range(8):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L += [f"s_mov_b32 s42, s{52 + j}", "s_swappc_b64 s[40:41], s[42:43]"]
        L.append("s_set_gpr_idx_off")
    elif mode in ("call1", "callidx0"):  # 8 calls per iteration, no M0 change (call1: no idx mode at all)
        if mode == "callidx0":
            L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        L += ["s_mov_b32 s43, s45"]
        for j in range(8):
            L += [f"s_bfe_u32 s42, {'s50' if j < 4 else 's51'}, {0x80000 + 8 * (j % 4)}", "s_lshl3_add_u32 s42, s42, s42",
                  "s_lshl3_add_u32 s42, s42, s44", "s_swappc_b64 s[40:41], s[42:43]"]
        if mode == "callidx0":
            L.append("s_set_gpr_idx_off")
    elif mode == "m0mov":  # as inline, M0 set by s_mov_b32 m0 instead of s_set_gpr_idx_idx
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_mov_b32 m0, {8 * j}")
            L += snippet(c, [])
        L.append("s_set_gpr_idx_off")
    elif mode in ("call64r", "call128r"):  # as call72r with 64- / 128-byte snippet slots
        stride = 64 if mode == "call64r" else 128
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j in range(8):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L += ["s_mul_i32 s49, s49, 0x41c64e6d", "s_add_u32 s49, s49, 12345",
                  "s_lshr_b32 s50, s49, 24", f"s_mul_i32 s50, s50, {stride}",
                  "s_add_u32 s42, s44, s50", "s_addc_u32 s43, s45, 0", "s_swappc_b64 s[40:41], s[42:43]"]
        L.append("s_set_gpr_idx_off")
    elif mode == "call72r":  # idx mode, one table, coefficient varies per call (s49 = LCG state)
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j in range(8):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L += ["s_mul_i32 s49, s49, 0x41c64e6d", "s_add_u32 s49, s49, 12345",
                  "s_lshr_b32 s50, s49, 24", "s_mul_i32 s50, s50, 72",
                  "s_add_u32 s42, s44, s50", "s_addc_u32 s43, s45, 0", "s_swappc_b64 s[40:41], s[42:43]"]
        L.append("s_set_gpr_idx_off")
    elif mode in ("call4r", "call2r"):  # no idx mode: 4 / 2 tables, 8 products cycle over them
        nt = 4 if mode == "call4r" else 2
        for j in range(8):
            L += ["s_mul_i32 s49, s49, 0x41c64e6d", "s_add_u32 s49, s49, 12345",
                  "s_lshr_b32 s50, s49, 24", "s_mul_i32 s50, s50, 72",
                  f"s_add_u32 s50, s50, {(j % nt) * 257 * 72}",
                  "s_add_u32 s42, s44, s50", "s_addc_u32 s43, s45, 0", "s_swappc_b64 s[40:41], s[42:43]"]
    elif mode == "call8r":  # no idx mode: 8 tables (one per accumulator set), random coefficients
        for j in range(8):
            L += ["s_mul_i32 s49, s49, 0x41c64e6d", "s_add_u32 s49, s49, 12345",
                  "s_lshr_b32 s50, s49, 24", "s_mul_i32 s50, s50, 72",
                  f"s_add_u32 s50, s50, {j * 257 * 72}",
                  "s_add_u32 s42, s44, s50", "s_addc_u32 s43, s45, 0", "s_swappc_b64 s[40:41], s[42:43]"]
    elif mode == "direct":
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L.append(f"s_branch jp_direct_{j}")
            L.append(f"jp_direct_ret_{j}:")
        L.append("s_set_gpr_idx_off")
        L.append("s_branch jp_direct_end")
        for j, c in enumerate(COEF):
            L.append(".p2align 6")
            L.append(f"jp_direct_{j}:")
            L += snippet(c, [f"s_branch jp_direct_ret_{j}"])
        L.append("jp_direct_end:")
    elif mode == "setpc1":
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for j, c in enumerate(COEF):
            if j:
                L.append(f"s_set_gpr_idx_idx {8 * j}")
            L.append(f"s_add_u32 s42, s46, {128 * c}")
            L.append("s_addc_u32 s43, s47, 0")
            L.append("s_setpc_b64 s[42:43]")
            L.append(f"jp_s1_ret_{j}:")
            if j < 7:
                pass
        L.append("s_set_gpr_idx_off")
    return L


def kernel(mode):
    regs = ", ".join(f'"v{i}"' for i in range(ACC, 128)) + ', "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "m0"'
    b = body(mode)
    pre = []
    tables = []
    if mode == "call72":
        pre = ["s_getpc_b64 s[44:45]", "s_add_u32 s44, s44, jp_tab72@rel32@lo+4", "s_addc_u32 s45, s45, jp_tab72@rel32@hi+12"]
        tables = ["s_branch jp_t72_end"] + table("jp_tab72", 3, ["s_setpc_b64 s[40:41]"]) + ["jp_t72_end:"]
    if mode == "call128":
        pre = ["s_getpc_b64 s[44:45]", "s_add_u32 s44, s44, jp_tab128@rel32@lo+4", "s_addc_u32 s45, s45, jp_tab128@rel32@hi+12"]
        tables = ["s_branch jp_t128_end"] + table("jp_tab128", 7, ["s_setpc_b64 s[40:41]"]) + ["jp_t128_end:"]
    if mode in ("v2", "rl", "call1", "callidx0"):
        pre = ["s_getpc_b64 s[44:45]", "s_add_u32 s44, s44, jp_tab72" + mode + "@rel32@lo+4", "s_addc_u32 s45, s45, jp_tab72" + mode + "@rel32@hi+12",
               "s_mov_b32 s50, 0x8e1fca53", "s_mov_b32 s51, 0xd967b235"]
        if mode == "rl":
            pre += ["v_mbcnt_lo_u32_b32 v21, -1, 0", "v_mbcnt_hi_u32_b32 v21, -1, v21", "v_and_b32 v21, 7, v21",
                    "v_mul_u32_u24 v21, 41, v21", "v_and_b32 v21, 255, v21", "v_mul_u32_u24 v21, 72, v21",
                    "v_add_u32 v20, s44, v21"]
        tables = ["s_branch jp_t72e" + mode] + table("jp_tab72" + mode, 3, ["s_setpc_b64 s[40:41]", "s_nop 0"]) + ["jp_t72e" + mode + ":"]
    if mode in ("call64r", "call128r"):
        lab = "jp_tab" + mode
        pre = ["s_getpc_b64 s[44:45]", f"s_add_u32 s44, s44, {lab}@rel32@lo+4", f"s_addc_u32 s45, s45, {lab}@rel32@hi+12",
               "s_mov_b32 s49, 1"]
        t = ["s_branch " + lab + "_end", ".p2align 7", lab + ":"]
        for c in range(256):
            t.append(".p2align 6" if mode == "call64r" else ".p2align 7")
            v = c
            for bb in range(8):
                if bb == 7 and mode == "call64r":  # 7 bitop3 + one VOP2 xor + return = 64 bytes
                    t.append(f"v_xor_b32 v{ACC + bb}, v{T0 + (v & 15)}, v{ACC + bb}")
                else:
                    t.append(f"v_bitop3_b32 v{ACC + bb}, v{ACC + bb}, v{T0 + (v & 15)}, v{T1 + (v >> 4)} bitop3:0x96")
                v = gmul2(v)
            t.append("s_setpc_b64 s[40:41]")
        tables = t + [lab + "_end:"]
    if mode == "call72r":
        pre = ["s_getpc_b64 s[44:45]", "s_add_u32 s44, s44, jp_tab72r@rel32@lo+4", "s_addc_u32 s45, s45, jp_tab72r@rel32@hi+12",
               "s_mov_b32 s49, 1"]
        tables = ["s_branch jp_t72r_end"] + table("jp_tab72r", 3, ["s_setpc_b64 s[40:41]"]) + ["jp_t72r_end:"]
    if mode in ("call8r", "call4r", "call2r"):
        nt = {"call8r": 8, "call4r": 4, "call2r": 2}[mode]
        lab = f"jp_tab{nt}r"
        pre = ["s_getpc_b64 s[44:45]", f"s_add_u32 s44, s44, {lab}@rel32@lo+4", f"s_addc_u32 s45, s45, {lab}@rel32@hi+12",
               "s_mov_b32 s49, 1"]
        t8 = ["s_getpc_b64 s[52:53]", f"s_add_u32 s52, s52, {lab}_end@rel32@lo+4",
              f"s_addc_u32 s53, s53, {lab}_end@rel32@hi+12", "s_setpc_b64 s[52:53]", ".p2align 3", f"{lab}:"]
        for j in range(nt):
            for c in range(257):
                t8.append(".p2align 3")
                v = c if c < 256 else 0
                for bb in range(8):
                    t8.append(f"v_bitop3_b32 v{ACC + 8 * j + bb}, v{ACC + 8 * j + bb}, v{T0 + (v & 15)}, v{T1 + (v >> 4)} bitop3:0x96")
                    v = gmul2(v)
                t8.append("s_setpc_b64 s[40:41]")
        tables = t8 + [f"{lab}_end:"]
    if mode == "setpc1":
        # one table per call site is too big; use a single return via a per-site SGPR pair:
        # snippet ends with s_setpc_b64 s[40:41], the caller loads s[40:41] with its return
        # address by s_getpc before the jump (no s_swappc), i.e. still two redirects -- measures
        # the s_getpc+s_setpc form against s_swappc. s_getpc returns the address of the s_add that
        # follows it; the return lands after the s_setpc: s_add (4 B, inline constant) + s_addc (4) + s_setpc (4).
        b = ["s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)"]
        for j, c in enumerate(COEF):
            if j:
                b.append(f"s_set_gpr_idx_idx {8 * j}")
            b += [f"s_add_u32 s42, s46, {128 * c}", "s_addc_u32 s43, s47, 0", "s_getpc_b64 s[40:41]",
                  "s_add_u32 s40, s40, 12", "s_addc_u32 s41, s41, 0", "s_setpc_b64 s[42:43]"]
        b.append("s_set_gpr_idx_off")
        pre = ["s_getpc_b64 s[46:47]", "s_add_u32 s46, s46, jp_tabs1@rel32@lo+4", "s_addc_u32 s47, s47, jp_tabs1@rel32@hi+12"]
        tables = ["s_branch jp_ts1_end"] + table("jp_tabs1", 7, ["s_setpc_b64 s[40:41]"]) + ["jp_ts1_end:"]
    q = lambda ls: "\n".join(f'        "{l}\\n"' for l in ls)
    return f'''__global__ __launch_bounds__(256) void k_{mode}(unsigned long long *st, int iters) {{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile(
{q(pre + ["s_mov_b32 s48, 0"])}
        "jp_loop_{mode}:\\n"
{q(b)}
        "s_add_u32 s48, s48, 1\\n"
        "s_cmp_lt_u32 s48, %0\\n"
        "s_cbranch_scc1 jp_loop_{mode}\\n"
{q(tables)}
        :: "s"(iters) : {regs}, "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "v20", "v21", "scc", "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {{
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        st[4 * w] = t0; st[4 * w + 1] = t1; st[4 * w + 2] = r0; st[4 * w + 3] = r1;
    }}
}}
'''


MODES = ["noidx", "call72r", "call64r", "call128r", "v2"]


def main():
    src = ["// GENERATED by tools/jump_probe_gen.py -- measurement only, not part of the product.",
           "#include <hip/hip_runtime.h>", "#include <stdio.h>", "#include <stdlib.h>", "#include <string.h>",
           '#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\\n", hipGetErrorString(e_)); exit(1); } } while (0)']
    for m in MODES:
        src.append(kernel(m))
    src.append("typedef void (*kfn)(unsigned long long *, int);")
    src.append("struct V { const char *name; kfn f; };")
    src.append("static V vars[] = {" + ", ".join(f'{{"{m}", k_{m}}}' for m in MODES) + "};")
    src.append(r'''
// jump_probe BLOCKS_PER_CU ITERS   (8 products = 64 bitop3 per iteration per wave)
int main(int argc, char **argv) {
    const int bpc = argc > 1 ? atoi(argv[1]) : 4;
    const int iters = argc > 2 ? atoi(argv[2]) : 4000;
    const int nb = 256 * bpc, nw = nb * 4;
    unsigned long long *st, *h = (unsigned long long *)malloc(sizeof(unsigned long long) * 4 * nw);
    CK(hipMalloc(&st, sizeof(unsigned long long) * 4 * nw));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (auto &v : vars) {
        for (int pass = 0; pass < 3; ++pass) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.f, dim3(nb), dim3(256), 0, 0, st, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(h, st, sizeof(unsigned long long) * 4 * nw, hipMemcpyDeviceToHost));
            double cyc = 0, rt = 0;
            for (int w = 0; w < nw; ++w) { cyc += h[4 * w + 1] - h[4 * w]; rt += h[4 * w + 3] - h[4 * w + 2]; }
            cyc /= nw; rt /= nw;
            const double ghz = cyc / (rt * 10.0);
            const double products = (double)iters * 8 * bpc;  // per SIMD
            if (pass == 2)
                printf("%-8s waves/SIMD=%d %.3f ms clock %.2f GHz  SIMD-cycles per product: %.1f (bitop3: %.2f)\n",
                       v.name, bpc, ms, ghz, ms * 1e-3 * ghz * 1e9 / products, ms * 1e-3 * ghz * 1e9 / products / 8);
            fflush(stdout);
        }
    }
    return 0;
}
''')
    with open(os.path.join(ROOT, "tools", "jump_probe.hip"), "w") as f:
        f.write("\n".join(src) + "\n")


if __name__ == "__main__":
    main()
