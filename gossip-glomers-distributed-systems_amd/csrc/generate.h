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
// Rows [rlo, rhi) only (a vertex-sharded rank's own rows): row_ptr of rhi - rlo
// rows from 0, global column ids; the pair stream is generated whole, and
// the keys of other rows are never stored.
int build_csr_rows(const gg_gen_spec& s, hipStream_t st, uint32_t col_or, uint64_t rlo, uint64_t rhi, Csr* out,
                   std::string* err);
int max_degree(const int64_t* d_rp, uint64_t V, hipStream_t st, uint64_t* out, std::string* err);
// Rows by descending degree (ties by id), columns renumbered to the new rows
// (| col_or), each list kept in its original (ascending id) order; replaces g's
// arrays. gid_out: [rows] node id of each row (~0u padding); host copies of
// gid and of loc (node -> row).
int degree_reorder(Csr* g, uint64_t rows, hipStream_t st, uint32_t col_or, uint32_t** gid_out,
                   std::vector<uint32_t>* gid_host, std::vector<uint32_t>* loc_host, std::string* err);

// A vertex-sharded rank's exchange structures, built on the device from its
// own rows (g: build_csr_rows of [lo, hi), global columns; symmetric graphs).
// plo: [P+1] row ranges of the parts. On return g's columns are local rows
// (own rows from 0, ghosts from ghost0, | col_or); device arrays belong to the
// caller.
struct Shard {
    uint64_t n_ghost = 0, n_send = 0, n_cut = 0;
    std::vector<uint32_t> ghosts_host;        // [n_ghost] ghost node ids, ascending
    std::vector<uint64_t> send_off, recv_off; // [P+1] per peer part
    uint32_t* send_idx = nullptr;             // [n_send] owned rows, by part, ascending
    int64_t* gout_ptr = nullptr;              // [n_ghost+1] ghost -> owned receivers
    uint32_t* gout_col = nullptr;             // [n_cut]
    uint32_t* gout_sidx = nullptr;            // [n_cut] the receiver's send-list entry
    uint32_t* gid = nullptr;                  // [rows] node id of every local row (~0u padding)
};
int shard_csr(Csr* g, uint64_t lo, uint64_t hi, const std::vector<uint64_t>& plo, uint64_t ghost0, uint32_t col_or,
              hipStream_t st, Shard* out, std::string* err);
// A shard's local rows in locality order (the single engine's degree_reorder
// rule): owned rows by descending degree, ghost rows by descending count of
// owned receivers (the rows the shard's gathers hit most come first), ties by
// the old row. Renumbers g's columns, sh's gid (device and host), send_idx and
// ghost -> owned lists (re-indexed by the new ghost rows). Returns, on the
// device, grow[old ghost index] = new ghost index (the exchange still delivers
// ghosts in the sender's order, ascending id) and, on the host, own_row[old
// owned row] = new owned row.
int shard_reorder(Csr* g, Shard* sh, uint64_t ghost0, uint32_t col_or, hipStream_t st, uint32_t** grow_out,
                  std::vector<uint32_t>* own_row, std::string* err);

}  // namespace gg_gen

#endif
