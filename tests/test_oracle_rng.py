"""The oracle's std::mt19937 + uniform_int_distribution<int> restatement against libstdc++ itself (a few-line g++
program), for the draws the C++ LoopHandler's getFRANSAC makes: one engine seeded 0, a fresh distribution of range
[0, n - 1] per call (ya_vo_amd/frontend/loop_handler.cpp getFRANSAC; the reference's src/3DHandler.cc:157-164 seeds
from std::random_device)."""
import shutil
import subprocess

import numpy as np
import pytest

PROG = r"""
#include <cstdio>
#include <random>
int main() {
    std::mt19937 g(0);
    const int ns[] = {8, 9, 1935, 2000, 4096, 3, 1000000};
    for (int n : ns) {
        std::uniform_int_distribution<int> d(0, n - 1);
        for (int i = 0; i < 3200; ++i) std::printf("%d\n", d(g));
    }
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_mt19937_uniform_ints_match_libstdcxx(tmp_path, oracle):
    src = tmp_path / "draw.cc"
    src.write_text(PROG)
    exe = tmp_path / "draw"
    subprocess.run(["g++", "-O1", "-o", str(exe), str(src)], check=True)
    ref = np.array(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split(), np.int64)
    g = oracle.mt19937(0)
    got = np.concatenate([g.uniform_ints(0, n - 1, 3200) for n in (8, 9, 1935, 2000, 4096, 3, 1000000)])
    np.testing.assert_array_equal(got, ref)
