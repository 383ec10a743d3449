// gossip_host.h — host-side input builders (libgossip_host.so): topologies as
// CSR, the form gg_topology() consumes. See topology.cpp.
#ifndef GOSSIP_HOST_H_
#define GOSSIP_HOST_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t n_nodes;
    uint64_t nnz;
    int64_t* row_ptr; /* [n_nodes + 1], malloc'd */
    int32_t* col;     /* [nnz], malloc'd, rows ascending + unique */
} gg_csr;

void ggh_csr_free(gg_csr* c);
int ggh_tree(uint64_t V, uint32_t k, gg_csr* out);
int ggh_random_regular(uint64_t V, uint32_t d, uint64_t seed, gg_csr* out);
int ggh_rmat(uint64_t V, uint32_t edge_factor, double a, double b, double c, uint64_t seed,
             gg_csr* out);
int ggh_grid_links(uint64_t side, uint64_t seed, gg_csr* out);
int ggh_topology_json(const char* text, uint64_t len, gg_csr* out);
int ggh_is_symmetric(const int64_t* row_ptr, const int32_t* col, uint64_t V);
int ggh_components(const int64_t* row_ptr, const int32_t* col, uint64_t V, uint32_t* label);
int ggh_bfs(const int64_t* row_ptr, const int32_t* col, uint64_t V, uint32_t src, int32_t* dist);

#ifdef __cplusplus
}
#endif

#endif
