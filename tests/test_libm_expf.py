"""gs_libm.hpp's glibc_expf (used by the GPU load path) against the C library expf the
reference's loader calls (std::exp on float, src/Splats.cpp:318-326): bit-identical on a
prime-strided sample of all 2^32 float inputs plus the whole range where splat activations
live.  The full 2^32 sweep was run when the restatement was written (0 mismatches)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include <cmath>
#include <cstdio>
#include "gs_libm.hpp"
int main() {
    unsigned long long bad = 0, tot = 0;
    #pragma omp parallel for reduction(+:bad,tot) schedule(static)
    for (long long i = 0; i < (1LL << 32); i += 7) {          // every 7th bit pattern
        const uint32_t u = (uint32_t)i;
        float x; std::memcpy(&x, &u, 4);
        if (x != x) continue;
        ++tot;
        if (gs::libm_f2u(gs::glibc_expf(x)) != gs::libm_f2u(expf(x))) ++bad;
    }
    #pragma omp parallel for reduction(+:bad,tot) schedule(static)
    for (long long i = 0; i < (1LL << 24); ++i) {               // dense in [-20, 20]
        const float x = -20.0f + 40.0f * (float)i / (float)(1 << 24);
        ++tot;
        if (gs::libm_f2u(gs::glibc_expf(x)) != gs::libm_f2u(expf(x))) ++bad;
    }
    std::printf("%llu %llu\n", tot, bad);
    return 0;
}
'''


def test_glibc_expf_restatement(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = tmp_path / "t"
    inc = os.path.join(ROOT, "openglgaussiansplattingrenderer_amd", "csrc")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-I", inc, str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300).stdout.split()
    tot, bad = int(out[0]), int(out[1])
    assert tot > 600_000_000 and bad == 0, (tot, bad)
