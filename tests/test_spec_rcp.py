"""gg_sync_interval_rcp (the engine's timer form: the seed's mix and the
remainder's reciprocal precomputed) against gg_sync_interval, the spec
function O2 uses, on random and edge inputs: every jitter from 1 to 4096, the
largest jitters, node ids near 2^44 and timer counts near 2^32
(include/gossip_spec.h). Compiled with g++ from the shared header."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <cstdio>
#include <cstdint>
#include "gossip_spec.h"
int main() {
    uint64_t x = 0x1234567887654321ull, bad = 0, n = 0;
    auto rnd = [&]() { x = gg_mix64(x); return x; };
    auto check = [&](uint64_t seed, uint64_t v, uint32_t k, uint32_t base, uint32_t jit) {
        const uint32_t a = gg_sync_interval(seed, v, k, base, jit);
        const uint32_t b = gg_sync_interval_rcp(gg_mix64(seed ^ GG_TAG_SYNC), gg_sync_rcp(jit), v, k, base, jit);
        ++n;
        if (a != b && bad++ < 5) printf("differ: seed %llx v %llu k %u jitter %u: %u != %u\n",
                                        (unsigned long long)seed, (unsigned long long)v, k, jit, a, b);
    };
    for (uint32_t jit = 0; jit <= 4096; ++jit)
        for (int t = 0; t < 200; ++t) check(rnd(), rnd() >> 20, (uint32_t)rnd(), (uint32_t)rnd() % 100, jit);
    const uint32_t big[] = {42949672u, 42949673u, 1u << 31, 0xFFFFFFFFu, 0xFFFFFFFEu, 3000000000u, 65535u, 65536u};
    for (uint32_t jit : big)
        for (int t = 0; t < 200000; ++t) check(rnd(), rnd() >> 20, (uint32_t)rnd(), 20, jit);
    for (int t = 0; t < 2000000; ++t) check(rnd(), rnd() >> 20, (uint32_t)rnd(), 20, (uint32_t)rnd());
    for (int t = 0; t < 200000; ++t) check(rnd(), (1ull << 44) - 1 - (t & 7), 0xFFFFFFFFu - (t & 3), 20, 10);
    printf("%llu checked, %llu differ\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
"""


def test_sync_interval_rcp_equals_spec(tmp_path):
    src = tmp_path / "rcp.cpp"
    src.write_text(SRC)
    exe = tmp_path / "rcp"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert " 0 differ" in p.stdout
