// Host-side topology builders: the synthetic inputs of the five configs
//  as CSR adjacency, the form gg_topology() takes.
//
// The reference receives its topology from the Maelstrom harness as a JSON map
// `{"topology": {"n0": ["n1", ...], ...}}` and each node keeps its own row
// (HandleTopology, `broadcast/broadcast.go:36-48`, TopologyMsgBody `:18-20`).
// Maelstrom's `--topology tree4` is the 4-ary tree of config C1/C2. Every
// builder here returns rows that are ascending, unique and free of self loops,
// and symmetric (u lists v iff v lists u), as Maelstrom's topologies are.
//
// All randomness is splitmix64 of (seed, stream, index) so results are
// independent of thread count.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "gossip_spec.h"
#include "gossip_host.h"

namespace {

struct Rng {  // splitmix64 stream
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { return gg_mix64(s += 0x9E3779B97F4A7C15ull); }
    uint64_t below(uint64_t n) {  // unbiased enough for n << 2^64
        return (uint64_t)(((unsigned __int128)next() * n) >> 64);
    }
};

int n_threads() {
    unsigned hc = std::thread::hardware_concurrency();
    int t = hc ? (int)hc : 1;
    if (const char* s = getenv("GG_HOST_THREADS")) t = std::max(1, atoi(s));
    return std::min(t, 16);
}

template <class F>
void parallel_for(uint64_t n, F f) {
    int T = (int)std::min<uint64_t>((uint64_t)n_threads(), std::max<uint64_t>(1, n / 65536));
    if (T <= 1) { f(0, n, 0); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(f, n * t / T, n * (t + 1) / T, t);
    for (auto& x : th) x.join();
}

// Build a symmetric CSR from undirected pairs (each pair inserted both ways),
// dropping self loops and duplicates.
int build_sym_csr(uint64_t V, const std::vector<uint32_t>& a, const std::vector<uint32_t>& b,
                  gg_csr* out) {
    const uint64_t m = a.size();
    std::vector<int64_t> deg(V + 1, 0);
    for (uint64_t k = 0; k < m; ++k) {
        if (a[k] == b[k]) continue;
        deg[a[k] + 1]++;
        deg[b[k] + 1]++;
    }
    for (uint64_t v = 0; v < V; ++v) deg[v + 1] += deg[v];
    std::vector<uint32_t> tmp((size_t)deg[V]);
    {
        std::vector<int64_t> pos(deg.begin(), deg.end() - 1);
        for (uint64_t k = 0; k < m; ++k) {
            if (a[k] == b[k]) continue;
            tmp[pos[a[k]]++] = b[k];
            tmp[pos[b[k]]++] = a[k];
        }
    }
    // sort + unique each row, count
    std::vector<int64_t> cnt(V + 1, 0);
    parallel_for(V, [&](uint64_t lo, uint64_t hi, int) {
        for (uint64_t v = lo; v < hi; ++v) {
            auto bgn = tmp.begin() + deg[v], end = tmp.begin() + deg[v + 1];
            std::sort(bgn, end);
            cnt[v + 1] = std::unique(bgn, end) - bgn;
        }
    });
    for (uint64_t v = 0; v < V; ++v) cnt[v + 1] += cnt[v];
    const uint64_t nnz = (uint64_t)cnt[V];
    int64_t* rp = (int64_t*)malloc((V + 1) * sizeof(int64_t));
    int32_t* col = (int32_t*)malloc(std::max<uint64_t>(1, nnz) * sizeof(int32_t));
    if (!rp || !col) { free(rp); free(col); return -12; }
    memcpy(rp, cnt.data(), (V + 1) * sizeof(int64_t));
    parallel_for(V, [&](uint64_t lo, uint64_t hi, int) {
        for (uint64_t v = lo; v < hi; ++v)
            for (int64_t k = 0; k < cnt[v + 1] - cnt[v]; ++k) col[cnt[v] + k] = (int32_t)tmp[deg[v] + k];
    });
    out->n_nodes = V;
    out->nnz = nnz;
    out->row_ptr = rp;
    out->col = col;
    return 0;
}

std::vector<uint32_t> permutation(uint64_t V, uint64_t seed) {
    std::vector<uint32_t> p(V);
    for (uint64_t i = 0; i < V; ++i) p[i] = (uint32_t)i;
    Rng r(seed);
    for (uint64_t i = V; i > 1; --i) std::swap(p[i - 1], p[r.below(i)]);
    return p;
}

}  // namespace

extern "C" {

void ggh_csr_free(gg_csr* c) {
    if (!c) return;
    free(c->row_ptr);
    free(c->col);
    c->row_ptr = nullptr;
    c->col = nullptr;
}

// k-ary tree in BFS numbering: parent(i) = (i-1)/k (Maelstrom `tree4` for k=4).
int ggh_tree(uint64_t V, uint32_t k, gg_csr* out) {
    if (!out || V == 0 || V > 0x7fffffffull || k == 0) return -22;
    int64_t* rp = (int64_t*)malloc((V + 1) * sizeof(int64_t));
    const uint64_t nnz = 2 * (V - 1);
    int32_t* col = (int32_t*)malloc(std::max<uint64_t>(1, nnz) * sizeof(int32_t));
    if (!rp || !col) { free(rp); free(col); return -12; }
    rp[0] = 0;
    for (uint64_t i = 0; i < V; ++i) {
        uint64_t d = (i > 0);
        uint64_t c0 = i * k + 1;
        if (c0 < V) d += std::min<uint64_t>(k, V - c0);
        rp[i + 1] = rp[i] + (int64_t)d;
    }
    parallel_for(V, [&](uint64_t lo, uint64_t hi, int) {
        for (uint64_t i = lo; i < hi; ++i) {
            int64_t p = rp[i];
            if (i > 0) col[p++] = (int32_t)((i - 1) / k);
            for (uint64_t c = i * k + 1; c <= i * k + k && c < V; ++c) col[p++] = (int32_t)c;
        }
    });
    out->n_nodes = V;
    out->nnz = nnz;
    out->row_ptr = rp;
    out->col = col;
    return 0;
}

// Random d-regular-ish graph: d/2 seeded permutations pi_j, edges {v, pi_j(v)},
// symmetrized, self loops and duplicates dropped (degree <= d).
int ggh_random_regular(uint64_t V, uint32_t d, uint64_t seed, gg_csr* out) {
    if (!out || V == 0 || V > 0x7fffffffull || d < 2 || d % 2) return -22;
    std::vector<uint32_t> a, b;
    a.reserve(V * d / 2);
    b.reserve(V * d / 2);
    for (uint32_t j = 0; j < d / 2; ++j) {
        auto p = permutation(V, gg_mix64(seed ^ (0x52454755ull + j)));
        for (uint64_t v = 0; v < V; ++v) {
            a.push_back((uint32_t)v);
            b.push_back(p[v]);
        }
    }
    return build_sym_csr(V, a, b, out);
}

// R-MAT (Chakrabarti et al. 2004): V*edge_factor directed samples over a
// 2^ceil(log2 V) square, quadrant probabilities (a,b,c,1-a-b-c), endpoints >= V
// resampled, ids relabelled by a seeded permutation, then symmetrized.
int ggh_rmat(uint64_t V, uint32_t edge_factor, double pa, double pb, double pc, uint64_t seed,
             gg_csr* out) {
    if (!out || V < 2 || V > 0x7fffffffull || edge_factor == 0) return -22;
    uint32_t scale = 0;
    while ((1ull << scale) < V) ++scale;
    const uint64_t m = V * edge_factor;
    std::vector<uint32_t> a(m), b(m);
    const uint64_t ta = (uint64_t)(pa * 18446744073709551616.0);
    const uint64_t tb = (uint64_t)((pa + pb) * 18446744073709551616.0);
    const uint64_t tc = (uint64_t)((pa + pb + pc) * 18446744073709551616.0);
    parallel_for(m, [&](uint64_t lo, uint64_t hi, int) {
        for (uint64_t k = lo; k < hi; ++k) {
            Rng r(gg_mix64(seed ^ 0x524d4154ull) ^ gg_mix64(k));
            uint64_t u, v;
            do {
                u = v = 0;
                for (uint32_t s = 0; s < scale; ++s) {
                    uint64_t x = r.next();
                    uint64_t bu = 0, bv = 0;
                    if (x < ta) {
                    } else if (x < tb) {
                        bv = 1;
                    } else if (x < tc) {
                        bu = 1;
                    } else {
                        bu = bv = 1;
                    }
                    u = (u << 1) | bu;
                    v = (v << 1) | bv;
                }
            } while (u >= V || v >= V);
            a[k] = (uint32_t)u;
            b[k] = (uint32_t)v;
        }
    });
    auto p = permutation(V, gg_mix64(seed ^ 0x5045524dull));
    parallel_for(m, [&](uint64_t lo, uint64_t hi, int) {
        for (uint64_t k = lo; k < hi; ++k) {
            a[k] = p[a[k]];
            b[k] = p[b[k]];
        }
    });
    return build_sym_csr(V, a, b, out);
}

// side x side 4-neighbour grid plus one seeded long-range link per node
// (a small world: Kleinberg-style shortcuts, uniform target), symmetrized.
int ggh_grid_links(uint64_t side, uint64_t seed, gg_csr* out) {
    if (!out || side < 2) return -22;
    const uint64_t V = side * side;
    if (V > 0x7fffffffull) return -22;
    std::vector<uint32_t> a, b;
    a.reserve(3 * V);
    b.reserve(3 * V);
    for (uint64_t y = 0; y < side; ++y)
        for (uint64_t x = 0; x < side; ++x) {
            uint64_t v = y * side + x;
            if (x + 1 < side) { a.push_back((uint32_t)v); b.push_back((uint32_t)(v + 1)); }
            if (y + 1 < side) { a.push_back((uint32_t)v); b.push_back((uint32_t)(v + side)); }
            Rng r(gg_mix64(seed ^ 0x4c494e4bull) ^ gg_mix64(v));
            a.push_back((uint32_t)v);
            b.push_back((uint32_t)r.below(V));
        }
    return build_sym_csr(V, a, b, out);
}

// Weakly connected components (union-find with path halving): label[v] = the
// smallest node id of v's component. Test/measurement helper (size-independent
// properties of full-size runs: a message reaches exactly its source's component).
int ggh_components(const int64_t* rp, const int32_t* col, uint64_t V, uint32_t* label) {
    std::vector<uint32_t> p(V);
    for (uint64_t v = 0; v < V; ++v) p[v] = (uint32_t)v;
    auto find = [&](uint32_t x) {
        while (p[x] != x) {
            p[x] = p[p[x]];
            x = p[x];
        }
        return x;
    };
    for (uint64_t u = 0; u < V; ++u)
        for (int64_t k = rp[u]; k < rp[u + 1]; ++k) {
            uint32_t a = find((uint32_t)u), b = find((uint32_t)col[k]);
            if (a == b) continue;
            if (a < b) p[b] = a;
            else p[a] = b;
        }
    for (uint64_t v = 0; v < V; ++v) label[v] = find((uint32_t)v);
    return 0;
}

// Directed hop distance from src along the rows (dist -1 = unreachable).
int ggh_bfs(const int64_t* rp, const int32_t* col, uint64_t V, uint32_t src, int32_t* dist) {
    if (src >= V) return -22;
    for (uint64_t v = 0; v < V; ++v) dist[v] = -1;
    std::vector<uint32_t> cur{src}, nxt;
    dist[src] = 0;
    for (int32_t d = 1; !cur.empty(); ++d) {
        nxt.clear();
        for (uint32_t u : cur)
            for (int64_t k = rp[u]; k < rp[u + 1]; ++k) {
                const uint32_t w = (uint32_t)col[k];
                if (dist[w] < 0) {
                    dist[w] = d;
                    nxt.push_back(w);
                }
            }
        cur.swap(nxt);
    }
    return 0;
}

// Maelstrom `topology` message -> CSR (HandleTopology, broadcast/broadcast.go:36-48;
// TopologyMsgBody :18-20): accepts the whole body {"type":"topology",
// "topology":{"n0":["n1",...],...}} or just the map. Node "n<i>" is id i; V =
// 1 + the largest id named; a node without a row gets an empty list (:41-42);
// rows are sorted and de-duplicated (the engine's claim order is by id, not by
// list position). Returns -22 on malformed input.
int ggh_topology_json(const char* text, uint64_t len, gg_csr* out) {
    if (!text || !out) return -22;
    const char* p = text;
    const char* end = text + len;
    auto ws = [&]() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p; };
    auto lit = [&](char c) { ws(); if (p < end && *p == c) { ++p; return true; } return false; };
    auto str = [&](std::string& s) -> bool {
        ws();
        if (p >= end || *p != '"') return false;
        ++p;
        s.clear();
        while (p < end && *p != '"') {
            if (*p == '\\' && p + 1 < end) ++p;
            s.push_back(*p++);
        }
        if (p >= end) return false;
        ++p;
        return true;
    };
    auto node_id = [](const std::string& s, int64_t& id) -> bool {
        if (s.size() < 2 || s[0] != 'n') return false;
        id = 0;
        for (size_t k = 1; k < s.size(); ++k) {
            if (s[k] < '0' || s[k] > '9' || id > 0x7fffffff) return false;
            id = id * 10 + (s[k] - '0');
        }
        return id <= 0x7ffffffe;
    };
    // skip any JSON value (for the body's other keys)
    std::function<bool()> skip = [&]() -> bool {
        ws();
        if (p >= end) return false;
        if (*p == '"') { std::string t; return str(t); }
        if (*p == '{' || *p == '[') {
            const char close = *p == '{' ? '}' : ']';
            ++p;
            if (lit(close)) return true;
            do {
                if (close == '}') { std::string k; if (!str(k) || !lit(':')) return false; }
                if (!skip()) return false;
            } while (lit(','));
            return lit(close);
        }
        while (p < end && *p != ',' && *p != '}' && *p != ']') ++p;
        return true;
    };
    std::vector<std::pair<int64_t, std::vector<int64_t>>> rows;
    int64_t maxid = -1;
    auto parse_map = [&]() -> bool {  // {"n0": ["n1", ...], ...}
        if (!lit('{')) return false;
        if (lit('}')) return true;
        do {
            std::string k;
            int64_t u;
            if (!str(k) || !node_id(k, u) || !lit(':') || !lit('[')) return false;
            std::vector<int64_t> nb;
            if (!lit(']')) {
                do {
                    std::string t;
                    int64_t v;
                    if (!str(t) || !node_id(t, v)) return false;
                    nb.push_back(v);
                    maxid = std::max(maxid, v);
                } while (lit(','));
                if (!lit(']')) return false;
            }
            maxid = std::max(maxid, u);
            rows.emplace_back(u, std::move(nb));
        } while (lit(','));
        return lit('}');
    };
    // body or bare map: look for a "topology" key at the top level
    const char* save = p;
    bool ok = false;
    if (lit('{')) {
        std::string k;
        const char* key_at = p;
        if (str(k) && k.rfind("n", 0) == 0 && k.size() > 1 && k[1] >= '0' && k[1] <= '9') {
            p = save;
            ok = parse_map();
        } else {
            p = key_at;
            bool found = false;
            if (!lit('}')) {
                do {
                    if (!str(k) || !lit(':')) return -22;
                    if (k == "topology") {
                        if (!parse_map()) return -22;
                        found = true;
                    } else if (!skip()) {
                        return -22;
                    }
                } while (lit(','));
                if (!lit('}')) return -22;
            }
            ok = found;
        }
    }
    if (!ok) return -22;
    const uint64_t V = (uint64_t)(maxid + 1);
    std::vector<std::vector<int64_t>> adj(V);
    for (auto& r : rows) {
        auto& a = adj[r.first];
        a.insert(a.end(), r.second.begin(), r.second.end());
    }
    int64_t* rp = (int64_t*)malloc((V + 1) * sizeof(int64_t));
    uint64_t nnz = 0;
    for (auto& a : adj) {
        std::sort(a.begin(), a.end());
        a.erase(std::unique(a.begin(), a.end()), a.end());
        nnz += a.size();
    }
    int32_t* col = (int32_t*)malloc(std::max<uint64_t>(1, nnz) * sizeof(int32_t));
    if (!rp || !col) { free(rp); free(col); return -12; }
    rp[0] = 0;
    for (uint64_t v = 0; v < V; ++v) {
        for (uint64_t k = 0; k < adj[v].size(); ++k) col[rp[v] + k] = (int32_t)adj[v][k];
        rp[v + 1] = rp[v] + (int64_t)adj[v].size();
    }
    out->n_nodes = V;
    out->nnz = nnz;
    out->row_ptr = rp;
    out->col = col;
    return 0;
}

// Symmetric iff every edge u->v has v->u (rows ascending).
int ggh_is_symmetric(const int64_t* rp, const int32_t* col, uint64_t V) {
    for (uint64_t u = 0; u < V; ++u)
        for (int64_t k = rp[u]; k < rp[u + 1]; ++k) {
            uint64_t v = (uint64_t)col[k];
            if (!std::binary_search(col + rp[v], col + rp[v + 1], (int32_t)u)) return 0;
        }
    return 1;
}

}  // extern "C"
