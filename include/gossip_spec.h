/*
 * gossip_spec.h — the seeded functions of the determinization contract
 * (DESIGN.md §2), shared verbatim by the HIP engine, the C++ host code and the
 * CPU bitset oracle; oracle/o1_literal.py restates them independently in Python.
 *
 * They are part of the *input specification* (which round a node's sync timer
 * fires in, which side of a seeded bisection a node is on, how a round's node
 * sets are fingerprinted), not of the propagation algorithm under test.
 *
 * Reference anchors:
 *   sync interval  — `broadcast/main.go:44-50`: sleep(2 s + rand.Intn(1000) ms)
 *                    then SyncBroadcast(); with 100 ms ticks that is
 *                    base + floor(U[0,1000) / 100) ticks.
 *   bisection      — Maelstrom `--nemesis partition` (README.md:18), seeded.
 */
#ifndef GOSSIP_SPEC_H_
#define GOSSIP_SPEC_H_

#include <stdint.h>

#if defined(__HIPCC__)
#define GG_HD __host__ __device__ __forceinline__
#else
#define GG_HD static inline
#endif

#define GG_TAG_SYNC 0x53594e4353594e43ull /* "SYNCSYNC" */
#define GG_TAG_PART 0x5041525450415254ull /* "PARTPART" */
#define GG_TAG_HASH 0x4841534848415348ull /* "HASHHASH" */

/* splitmix64 finaliser (Steele, Lea, Flood 2014). */
GG_HD uint64_t gg_mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Ticks between the k-th and (k+1)-th firing of node v's sync timer
 * (k = 0 gives the first firing round T_1 = I(v,0); T_{k+1} = T_k + I(v,k)). */
GG_HD uint32_t gg_sync_interval(uint64_t seed, uint64_t v, uint32_t k, uint32_t base,
                                uint32_t jitter) {
    if (jitter == 0) return base;
    uint64_t h = gg_mix64(gg_mix64(seed ^ GG_TAG_SYNC) ^ gg_mix64((v << 20) ^ (uint64_t)k));
    return base + (uint32_t)((h % (100ull * jitter)) / 100ull);
}

/* High 64 bits of a 64 x 64-bit product. */
GG_HD uint64_t gg_umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

/* gg_sync_interval with the per-run constants precomputed: seedmix =
 * gg_mix64(seed ^ GG_TAG_SYNC) and rcp = floor((2^64 - 1) / m), m = 100 * jitter
 * (gg_sync_rcp). Bit-identical: q = floor(h * rcp / 2^64) is floor(h / m) or one
 * less, since h/m - h*rcp/2^64 = h (1 + s) / (m 2^64) < 1 with s = (2^64 - 1) mod m
 * < m; so h - q m < 2m and one subtraction gives h mod m. The device's timers
 * take this form (a 64-bit remainder by a run-time divisor is a long
 * instruction sequence on the GPU, paid by every wave holding a firing node). */
GG_HD uint64_t gg_sync_rcp(uint32_t jitter) {
    return jitter ? ~0ull / (100ull * jitter) : 0ull;
}

GG_HD uint32_t gg_sync_interval_rcp(uint64_t seedmix, uint64_t rcp, uint64_t v, uint32_t k,
                                    uint32_t base, uint32_t jitter) {
    if (jitter == 0) return base;
    const uint64_t m = 100ull * jitter;
    const uint64_t h = gg_mix64(seedmix ^ gg_mix64((v << 20) ^ (uint64_t)k));
    uint64_t r = h - gg_umulhi64(h, rcp) * m;
    if (r >= m) r -= m;
    return base + (uint32_t)(r < (1ull << 32) ? (uint32_t)r / 100u : r / 100ull);
}

/* Side (0/1) of node v in the seeded bisection of one partition window. */
GG_HD uint32_t gg_part_group(uint64_t seed, uint64_t epoch_seed, uint64_t v) {
    return (uint32_t)(gg_mix64(gg_mix64(seed ^ GG_TAG_PART ^ epoch_seed) ^ v) & 1ull);
}

/* Contribution to seen_hash of one set word that gained bits in a round:
 * word = the round's new bits of node v's word j, idx = v * (W/64) + j.
 * seen_hash = sum (mod 2^64) over all rounds so far and all such words. */
GG_HD uint64_t gg_word_hash(uint64_t idx, uint64_t word) {
    return gg_mix64(gg_mix64(idx ^ GG_TAG_HASH) ^ word);
}

#endif /* GOSSIP_SPEC_H_ */
