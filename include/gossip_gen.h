/*
 * gossip_gen.h — on-device topology generators of libgossip_hip.so
 * ("on-device graph generators ... for 10^9-node inputs").
 *
 * The reference receives its topology as one JSON `topology` message per node
 * (HandleTopology, `broadcast/broadcast.go:36-48`; TopologyMsgBody `:18-20`),
 * built by the Maelstrom harness (`--topology tree4` etc.). gg_topology() takes
 * that adjacency as a host CSR; for the synthetic configs of BASELINE.json the
 * CSR of a 10^9-node graph takes minutes to build on the host and tens of
 * seconds to upload. gg_topology_generate() builds the same
 * graph directly in HBM and installs it exactly as gg_topology() would.
 *
 * The graphs are DEFINED by the host builders of gossip_host.h (ggh_tree,
 * ggh_random_regular, ggh_rmat, ggh_grid_links — same seeds, same sampling
 * streams, same symmetrize + dedup rule): the generated CSR is bit-identical
 * to theirs (tests/test_gpu_generate.py). All generated graphs are symmetric.
 *
 * Only the HIP library exports these entry points (the CPU oracle takes the
 * host builders' CSR through gg_topology). A single engine (world == 1) keeps
 * the graph in HBM end to end; a sharded engine builds it on its device, then
 * copies it to the host for gg_topology's partition step (locality order,
 * ghosts, send lists), so no rank runs the host generator.
 */
#ifndef GOSSIP_GEN_H_
#define GOSSIP_GEN_H_

#include <stdint.h>

#include "gossip.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    GG_GEN_TREE = 1,           /* ggh_tree(n, k): k-ary tree, BFS numbering (Maelstrom tree<k>) */
    GG_GEN_RANDOM_REGULAR = 2, /* ggh_random_regular(n, k, seed): k/2 seeded permutations */
    GG_GEN_RMAT = 3,           /* ggh_rmat(n, k = edge factor, a, b, c, seed) */
    GG_GEN_GRID_LINKS = 4      /* ggh_grid_links(side = n, seed): n*n grid + 1 long link/node */
};

typedef struct {
    uint32_t kind; /* GG_GEN_* */
    uint32_t k;    /* tree arity | regular degree (even) | R-MAT edge factor | unused */
    uint64_t n;    /* nodes | grid side (nodes = n*n) */
    double a, b, c; /* R-MAT quadrant probabilities (d = 1 - a - b - c) */
    uint64_t seed; /* graph seed (not the engine's protocol seed) */
} gg_gen_spec;

/* Build the spec's graph on the engine's device and install it as the
 * topology (same effect as gg_topology with the host builder's CSR). The
 * graph's node count must equal the engine's n_nodes. *nnz_out (optional)
 * receives the number of directed adjacency entries. */
int gg_topology_generate(gg_engine* e, const gg_gen_spec* spec, uint64_t* nnz_out);

/* Copy the installed topology back as CSR (single engine only): row v = the nodes
 * that send to v, ascending — for a symmetric topology, topology[v] itself.
 * row_ptr has n_nodes + 1 entries; col holds cap entries (GG_EINVAL if the
 * graph has more; *nnz_out is set either way). col may be NULL to query nnz. */
int gg_topology_export(gg_engine* e, int64_t* row_ptr, int32_t* col, uint64_t cap, uint64_t* nnz_out);

#ifdef __cplusplus
}
#endif

#endif /* GOSSIP_GEN_H_ */
