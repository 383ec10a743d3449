// generate.h — internal interface between engine.hip and generate.hip.
#ifndef GG_GENERATE_H_
#define GG_GENERATE_H_

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "gossip_gen.h"

namespace gg_gen {

struct Csr {  // device CSR; the caller owns (hipFree) both arrays
    int64_t* row_ptr;
    uint32_t* col;  // column | col_or
    uint64_t V, nnz;
};

uint64_t spec_nodes(const gg_gen_spec& s);
// Build the spec's symmetric CSR on the current device (0 or a negative errno).
int build_csr(const gg_gen_spec& s, hipStream_t st, uint32_t col_or, Csr* out, std::string* err);
int max_degree(const int64_t* d_rp, uint64_t V, hipStream_t st, uint64_t* out, std::string* err);
// Rows by descending degree (ties by id), columns renumbered to the new rows
// (| col_or), each list kept in its original (ascending id) order; replaces g's
// arrays. gid_out: [rows] node id of each row (~0u padding); host copies of
// gid and of loc (node -> row).
int degree_reorder(Csr* g, uint64_t rows, hipStream_t st, uint32_t col_or, uint32_t** gid_out,
                   std::vector<uint32_t>* gid_host, std::vector<uint32_t>* loc_host, std::string* err);

}  // namespace gg_gen

#endif
