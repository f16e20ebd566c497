#!/usr/bin/env python3
"""Phase timing of rs_dec1_k (diagnostic, not part of the product): builds a
copy of libpoporon_amd/csrc/rs_single.hip with s_memtime stamps after each
phase (the `// STAMP n` markers are rewritten into stamp stores in the copy),
runs it on one 16-error codeword many times and prints the average cycles per
phase and the shader clock.  python tools/probes/dec1_phases.py"""
import ctypes as C
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "libpoporon_amd", "csrc", "rs_single.hip")

HARNESS = r'''
extern "C" int probe_run(int reps, unsigned long long *out, int nst, int *okp, int *corp) {
    RsDevTables *T; hipMalloc(&T, sizeof(RsDevTables));
    static RsDevTables h; memset(&h, 0, sizeof(h));
    unsigned x = 1; unsigned char lg[256]; lg[0] = 255;
    for (int i = 0; i < 255; i++) { h.exp2[i] = x; lg[x] = i; x <<= 1; if (x & 256) x ^= 0x11D; }
    for (int i = 255; i < 511; i++) h.exp2[i] = h.exp2[i - 255];
    h.exp2[511] = 0; memcpy(h.log, lg, 256);
    hipMemcpy(T, &h, sizeof(h), hipMemcpyHostToDevice);
    /* generator (log form) and one encoded codeword of data[i] = i*7+3 */
    unsigned g[33] = {1};
    for (int i = 0; i < 32; i++) { /* g *= (x + alpha^(1+i)) */
        unsigned r = h.exp2[1 + i];
        for (int j = i + 1; j > 0; j--) {
            unsigned p = 0;
            if (g[j] ) p = h.exp2[(lg[g[j]] + lg[r]) % 255];
            g[j] = g[j - 1] ^ p;
        }
        g[0] = h.exp2[(lg[g[0]] + lg[r]) % 255];
    }
    unsigned char cw[255];
    for (int i = 0; i < 223; i++) cw[i] = (unsigned char)(i * 7 + 3);
    unsigned char par[32] = {0};
    for (int i = 0; i < 223; i++) {
        unsigned fb = cw[i] ^ par[0];
        memmove(par, par + 1, 31); par[31] = 0;
        if (fb) for (int j = 0; j < 32; j++) if (g[31 - j]) par[j] ^= h.exp2[(lg[fb] + lg[g[31 - j]]) % 255];
    }
    memcpy(cw + 223, par, 32);
    unsigned char bad[255]; memcpy(bad, cw, 255);
    for (int k = 0; k < 16; k++) bad[(k * 37 + 5) % 255] ^= (unsigned char)(k * 13 + 1);
    unsigned char *d; hipMalloc(&d, 1024);
    unsigned long long *st; hipMalloc(&st, 64 * 8);
    RsCorrParams P; memset(&P, 0, sizeof(P)); P.fcr = 1; P.prim = 1; P.iprim = 1; P.size = 223; P.pad = 0; P.vfast = 1;
    unsigned long long acc[64] = {0};
    for (int r = 0; r < reps; r++) {
        hipMemcpy(d, bad, 255, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(rs_dec1_k, dim3(1), dim3(256), 0, 0, T, P, 0u, d, d + 223, nullptr, nullptr, nullptr, 0u,
                           nullptr, d + 600, d + 601, nullptr, 0u, st);
        hipDeviceSynchronize();
        unsigned long long hs[64]; hipMemcpy(hs, st, 64 * 8, hipMemcpyDeviceToHost);
        if (r >= 10) for (int i = 0; i < nst; i++) acc[i] += hs[i];
    }
    unsigned char res[255 + 2]; hipMemcpy(res, d, 255, hipMemcpyDeviceToHost); hipMemcpy(res + 255, d + 600, 2, hipMemcpyDeviceToHost);
    *okp = res[255] | (memcmp(res, cw, 255) == 0 ? 2 : 0); *corp = res[256];
    for (int i = 0; i < nst; i++) out[i] = acc[i] / (reps - 10);
    return 0;
}
'''


def main():
    src = open(SRC).read()
    n = 0

    def stamp(m):
        nonlocal n
        k = int(m.group(1))
        n = max(n, k + 1)
        return (f"if (threadIdx.x == 0) {{ __builtin_amdgcn_s_waitcnt(0); stamps_[{2*k}] = __builtin_amdgcn_s_memtime(); "
                f"stamps_[{2*k+1}] = __builtin_amdgcn_s_memrealtime(); }}")
    src = re.sub(r"/\* STAMP (\d+) \*/", stamp, src)
    src = src.replace("uint32_t *flag, uint32_t seq)\n{\n    __shared__ Dec1Smem s;",
                      "uint32_t *flag, uint32_t seq, unsigned long long *stamps_)\n{\n    __shared__ Dec1Smem s;")
    src = src[:src.index("/* ------------------------------------------------------------------------ */\n/* launchers")]
    bdir = os.path.join(ROOT, "tools", "probes", "_build")
    so = os.path.join(bdir, "dec1_phases.so")
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        os.makedirs(bdir, exist_ok=True)
        with tempfile.TemporaryDirectory() as td:
            f = os.path.join(td, "p.hip")
            open(f, "w").write("#include <cstring>\n" + src + HARNESS)
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                                   "-shared", "-w", "-I" + os.path.join(ROOT, "include"),
                                   "-I" + os.path.join(ROOT, "libpoporon_amd", "csrc"), "-o", so, f])
        print("built", n, "stamps")
        return
    if True:
        lib = C.CDLL(so)
        out = (C.c_ulonglong * 64)()
        ok, cor = C.c_int(0), C.c_int(0)
        lib.probe_run(2000, out, 2 * n, C.byref(ok), C.byref(cor))
        print("ok/restored", ok.value, "corrected", cor.value)
        t0, r0 = out[0], out[1]
        for k in range(1, n):
            dt = out[2 * k] - out[2 * (k - 1)]
            dr = out[2 * k + 1] - out[2 * (k - 1) + 1]
            print(f"phase {k}: {dt:8d} cycles  {dr / 100:8.2f} us")
        tot = out[2 * (n - 1)] - t0
        totr = out[2 * (n - 1) + 1] - r0
        print(f"total {tot} cycles {totr / 100:.2f} us  clock {tot / (totr / 100) / 1e3:.2f} GHz")


if __name__ == "__main__":
    main()
