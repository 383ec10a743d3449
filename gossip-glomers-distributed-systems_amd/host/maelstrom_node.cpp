// maelstrom_node.cpp — the Maelstrom JSON-lines handler surface of the
// reference's broadcast node (`broadcast/main.go:17-56`), served for EVERY node
// of the cluster by one process over the engine's C ABI.
//
// The reference is one OS process per node: Maelstrom pipes JSON messages
// {"src","dest","body"} to each, and node-to-node gossip crosses the network.
// Here the nodes are simulated in lockstep by the engine (libgossip_hip.so),
// so only client traffic crosses stdin/stdout:
//   init       -> init_ok      (node ids; the node count V)
//   topology   -> topology_ok  (HandleTopology `broadcast.go:36-48`; the first
//                               map builds the engine's CSR, later copies of the
//                               same map are acknowledged)
//   broadcast  -> broadcast_ok (HandleBroadcast from a client `:59-79`: the value
//                               is scheduled for the current round)
//   read       -> read_ok      (HandleRead `:124-132`: the node's values,
//                               ascending, including client broadcasts it got
//                               since the last round, as the reference's map
//                               holds them at once)
//   broadcast_ok               ignored (`main.go:38-40`)
//   tick {"rounds": k}         front-end extension: run k 100 ms rounds
//                               (lockstep mode, --tick-ms 0)
// Any other type: "No handler for <msg>" on stderr and exit status 1, as the
// pinned maelstrom library does. A handler that fails (e.g. the engine refuses a
// broadcast) answers with a Maelstrom error body {"code":13,"text":...} and the
// process keeps serving, as the library does when a handler returns an error.
//
// Values are unbounded, as the reference's map (`broadcast.go:14,73`): each
// engine holds --lanes values, and when every lane of the newest engine is in
// use a further engine over the same topology takes the new values. Values
// never interact (each one's propagation depends on no other value), so a read
// is the union of the node's sets over the engines — exactly one engine with
// every value. An older engine whose values can no longer change (symmetric
// topology, a round without deliveries, no client broadcast queued for it:
// every node then holds every value of its component) stops stepping until a
// client re-broadcasts one of its values. With --tick-ms T > 0 the process runs one
// round every T ms of wall time between input lines (Maelstrom --latency 100
// is one round per 100 ms).
//
// The engine library is loaded at run time (--engine PATH; default the HIP
// engine next to this binary), so the same front end drives the CPU oracle in
// the tests. There is no fallback: a missing or failing engine is an error.
#include <dlfcn.h>
#include <poll.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <unordered_map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "gossip.h"

namespace {

// ---- minimal JSON DOM -------------------------------------------------------
struct Json {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    int64_t inum = 0;
    bool integral = false;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;

    const Json* get(const char* key) const {
        if (kind != OBJ) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

struct Parser {
    const char* p;
    const char* end;
    void ws() {
        while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p;
    }
    bool lit(char c) {
        ws();
        if (p < end && *p == c) {
            ++p;
            return true;
        }
        return false;
    }
    bool string(std::string& s) {
        ws();
        if (p >= end || *p != '"') return false;
        ++p;
        s.clear();
        while (p < end && *p != '"') {
            if (*p == '\\' && p + 1 < end) {
                ++p;
                switch (*p) {
                    case 'n': s.push_back('\n'); break;
                    case 't': s.push_back('\t'); break;
                    case 'r': s.push_back('\r'); break;
                    case 'b': s.push_back('\b'); break;
                    case 'f': s.push_back('\f'); break;
                    case 'u': {  // keep ASCII, replace the rest
                        if (end - p < 5) return false;
                        const unsigned v = (unsigned)strtoul(std::string(p + 1, p + 5).c_str(), nullptr, 16);
                        s.push_back(v < 0x80 ? (char)v : '?');
                        p += 4;
                        break;
                    }
                    default: s.push_back(*p);
                }
                ++p;
            } else {
                s.push_back(*p++);
            }
        }
        if (p >= end) return false;
        ++p;
        return true;
    }
    bool value(Json& v) {
        ws();
        if (p >= end) return false;
        if (*p == '"') {
            v.kind = Json::STR;
            return string(v.str);
        }
        if (*p == '{') {
            ++p;
            v.kind = Json::OBJ;
            if (lit('}')) return true;
            do {
                std::string k;
                Json x;
                if (!string(k) || !lit(':') || !value(x)) return false;
                v.obj.emplace_back(std::move(k), std::move(x));
            } while (lit(','));
            return lit('}');
        }
        if (*p == '[') {
            ++p;
            v.kind = Json::ARR;
            if (lit(']')) return true;
            do {
                Json x;
                if (!value(x)) return false;
                v.arr.push_back(std::move(x));
            } while (lit(','));
            return lit(']');
        }
        if (end - p >= 4 && !strncmp(p, "true", 4)) {
            v.kind = Json::BOOL;
            v.b = true;
            p += 4;
            return true;
        }
        if (end - p >= 5 && !strncmp(p, "false", 5)) {
            v.kind = Json::BOOL;
            p += 5;
            return true;
        }
        if (end - p >= 4 && !strncmp(p, "null", 4)) {
            p += 4;
            return true;
        }
        const char* q = p;
        while (q < end && (strchr("+-.eE", *q) || (*q >= '0' && *q <= '9'))) ++q;
        if (q == p) return false;
        const std::string t(p, q);
        v.kind = Json::NUM;
        v.num = strtod(t.c_str(), nullptr);
        v.integral = t.find_first_of(".eE") == std::string::npos;
        if (v.integral) v.inum = strtoll(t.c_str(), nullptr, 10);
        p = q;
        return true;
    }
};

bool parse_json(const std::string& text, Json& out) {
    Parser ps{text.data(), text.data() + text.size()};
    if (!ps.value(out)) return false;
    ps.ws();
    return ps.p == ps.end;
}

void quote(std::string& o, const std::string& s) {
    o.push_back('"');
    for (char c : s) {
        if (c == '"' || c == '\\') {
            o.push_back('\\');
            o.push_back(c);
        } else if (c == '\n') {
            o += "\\n";
        } else {
            o.push_back(c);
        }
    }
    o.push_back('"');
}

// "n<i>" -> i, or -1
int64_t node_index(const std::string& s) {
    if (s.size() < 2 || s[0] != 'n') return -1;
    int64_t id = 0;
    for (size_t k = 1; k < s.size(); ++k) {
        if (s[k] < '0' || s[k] > '9' || id > 0x7fffffff) return -1;
        id = id * 10 + (s[k] - '0');
    }
    return id <= 0x7ffffffe ? id : -1;
}

// ---- the engine, loaded at run time ----------------------------------------
struct Api {
    void* h = nullptr;
    decltype(&gg_create) create = nullptr;
    decltype(&gg_destroy) destroy = nullptr;
    decltype(&gg_last_error) last_error = nullptr;
    decltype(&gg_topology) topology = nullptr;
    decltype(&gg_broadcast) broadcast = nullptr;
    decltype(&gg_step) step = nullptr;
    decltype(&gg_current_round) current_round = nullptr;
    decltype(&gg_read) read = nullptr;

    bool load(const std::string& path, std::string& err) {
        h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            err = dlerror();
            return false;
        }
#define GG_SYM(field, name)                                           \
    field = reinterpret_cast<decltype(field)>(dlsym(h, #name));       \
    if (!field) {                                                     \
        err = std::string("missing symbol ") + #name + " in " + path; \
        return false;                                                 \
    }
        GG_SYM(create, gg_create)
        GG_SYM(destroy, gg_destroy)
        GG_SYM(last_error, gg_last_error)
        GG_SYM(topology, gg_topology)
        GG_SYM(broadcast, gg_broadcast)
        GG_SYM(step, gg_step)
        GG_SYM(current_round, gg_current_round)
        GG_SYM(read, gg_read)
#undef GG_SYM
        return true;
    }
};

struct Options {
    std::string engine;
    uint32_t lanes = 1024;
    uint64_t seed = 0x6A09E667F3BCC909ull;
    bool sync = true;
    uint32_t batch = 0;  // gg_config.batch_ticks (0: the reference's per-value gossip)
    int device = 0;
    int tick_ms = 100;
    bool log = false;
};

class Front {
public:
    Front(const Options& o, Api& api) : opt_(o), api_(api) {}
    ~Front() {
        for (auto& x : engines_) api_.destroy(x.e);
    }

    // one input line; returns false to stop (exit status in *status)
    bool handle(const std::string& line, int* status) {
        Json msg;
        if (!parse_json(line, msg) || msg.kind != Json::OBJ) {
            fprintf(stderr, "malformed message: %s\n", line.c_str());
            *status = 1;
            return false;
        }
        const Json* src = msg.get("src");
        const Json* dest = msg.get("dest");
        const Json* body = msg.get("body");
        const Json* type = body ? body->get("type") : nullptr;
        if (!body || !type || type->kind != Json::STR) {
            fprintf(stderr, "No handler for %s\n", line.c_str());
            *status = 1;
            return false;
        }
        const std::string s = src && src->kind == Json::STR ? src->str : "";
        const std::string d = dest && dest->kind == Json::STR ? dest->str : "";
        const Json* mid = body->get("msg_id");
        const int64_t msg_id = mid && mid->kind == Json::NUM ? mid->inum : 0;
        const std::string& t = type->str;
        if (opt_.log) fprintf(stderr, "Received %s\n", line.c_str());
        if (t == "init") {
            if (const Json* ids = body->get("node_ids"))
                for (const auto& x : ids->arr) n_nodes_ = std::max<int64_t>(n_nodes_, node_index(x.str) + 1);
            if (const Json* id = body->get("node_id")) n_nodes_ = std::max<int64_t>(n_nodes_, node_index(id->str) + 1);
            return reply(d, s, msg_id, "init_ok", "", status);
        }
        if (t == "topology") {
            const Json* top = body->get("topology");
            if (!top || top->kind != Json::OBJ) return fail("topology without a map", status);
            if (engines_.empty() && !build(*top, status)) return false;
            return reply(d, s, msg_id, "topology_ok", "", status);
        }
        if (t == "broadcast") {
            const Json* m = body->get("message");
            if (!m || m->kind != Json::NUM || !m->integral) return fail("broadcast without an integer message", status);
            const int64_t v = node_index(d);
            if (v < 0) return fail("broadcast to a non-node " + d, status);
            if (!engines_.empty() && v >= V_) return error_reply(d, s, msg_id, "broadcast to an unknown node " + d);
            if (engines_.empty() && !build(Json{}, status)) return false;  // no topology yet: no neighbours
            if (s.empty() || s[0] != 'n') {  // from a client: the engine schedules it for this round
                std::string why;
                if (!client_broadcast((uint32_t)v, m->inum, why)) return error_reply(d, s, msg_id, why);
                pending_[(uint32_t)v].push_back(m->inum);
            }
            return reply(d, s, msg_id, "broadcast_ok", "", status);
        }
        if (t == "read") {
            const int64_t v = node_index(d);
            if (v < 0) return fail("read at a non-node " + d, status);
            if (engines_.empty() && !build(Json{}, status)) return false;
            std::vector<int64_t> vals;
            for (auto& x : engines_) {  // the union over the engines (disjoint value sets)
                std::vector<int64_t> part(64);
                uint64_t n = 0;
                int rc = api_.read(x.e, (uint32_t)v, part.data(), part.size(), &n);
                if (rc == 0 && n > part.size()) {
                    part.resize(n);
                    rc = api_.read(x.e, (uint32_t)v, part.data(), part.size(), &n);
                }
                if (rc) return error_reply(d, s, msg_id, std::string("gg_read: ") + api_.last_error(x.e));
                vals.insert(vals.end(), part.begin(), part.begin() + (std::ptrdiff_t)n);
            }
            auto it = pending_.find((uint32_t)v);  // client broadcasts not yet run through a round
            if (it != pending_.end()) vals.insert(vals.end(), it->second.begin(), it->second.end());
            std::sort(vals.begin(), vals.end());
            vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
            // ReadResponse.Messages starts as a nil slice (broadcast.go:125): an
            // empty read marshals as null, not []
            std::string extra = ",\"messages\":";
            if (vals.empty()) extra += "null";
            for (size_t k = 0; k < vals.size(); ++k) {
                extra.push_back(k ? ',' : '[');
                extra += std::to_string(vals[k]);
            }
            if (!vals.empty()) extra.push_back(']');
            return reply(d, s, msg_id, "read_ok", extra, status);
        }
        if (t == "broadcast_ok") return true;  // main.go:38-40
        if (t == "tick") {
            const Json* k = body->get("rounds");
            const int64_t n = k && k->kind == Json::NUM ? k->inum : 1;
            return run_rounds(n > 0 ? (uint32_t)n : 0u, status);
        }
        fprintf(stderr, "No handler for %s\n", line.c_str());
        *status = 1;
        return false;
    }

    bool run_rounds(uint32_t n, int* status) {
        if (engines_.empty() || !n) return true;
        std::vector<gg_round_stats> st(n);
        for (size_t k = 0; k < engines_.size(); ++k) {
            Slot& x = engines_[k];
            if (x.frozen) continue;
            const int rc = api_.step(x.e, n, st.data());
            if (rc) return fail(std::string("gg_step: ") + api_.last_error(x.e), status);
            // an older engine (no new values) on a symmetric topology whose last round
            // delivered nothing and that has no queued broadcast is final; batched
            // (--batch B): B + 1 quiet rounds in a row, so the last batch sent has
            // been delivered without news and nothing is pending
            uint32_t run = 0;
            while (run < n && st[n - 1 - run].new_bits == 0) ++run;
            x.quiet_run = run == n ? x.quiet_run + n : run;
            x.queued = false;
            x.frozen = can_freeze() && k + 1 < engines_.size() && x.quiet_run >= (opt_.batch ? opt_.batch + 1 : 1);
        }
        pending_.clear();
        round_ += n;
        return true;
    }

    size_t engine_count() const { return engines_.size(); }

    // Freezing an engine after a quiet round is safe only while every message is
    // delivered: on a symmetric topology each node then holds every value of its
    // component, so sync rounds can only repair losses and there are none. This
    // front end installs no partition windows and drops nothing (the simulated
    // network is Maelstrom's); a windowed engine would need its sync rounds to heal
    // a cut, and a frozen one would answer reads with stale sets.
    bool can_freeze() const { return sym_ && !windows_; }

private:
    struct Slot {
        gg_engine* e = nullptr;
        bool frozen = false;
        bool queued = false;  // a client broadcast waits for the next round
        uint32_t quiet_run = 0;  // rounds in a row without a delivery
    };

    // the engine that holds `value` (a new value: the newest engine, or a new one
    // when its lanes are all in use), scheduled for this round
    bool client_broadcast(uint32_t node, int64_t value, std::string& why) {
        auto it = owner_.find(value);
        size_t k = it != owner_.end() ? it->second : engines_.size() - 1;
        // a frozen engine sat out rounds at its fixed point: step it to the
        // current round first (nothing changes there, but batched gossip's send
        // ticks and the sync timers follow the round number)
        const int64_t behind = round_ - api_.current_round(engines_[k].e);
        if (behind > 0 && api_.step(engines_[k].e, (uint32_t)behind, nullptr)) {
            why = std::string("gg_step: ") + api_.last_error(engines_[k].e);
            return false;
        }
        int rc = api_.broadcast(engines_[k].e, node, value, round_);
        if (rc == GG_ENOSPC && it == owner_.end()) {
            if (!add_engine(why)) return false;
            k = engines_.size() - 1;
            engines_[k - 1].frozen = false;  // it may freeze at its next quiet round
            rc = api_.broadcast(engines_[k].e, node, value, round_);
        }
        if (rc) {
            why = std::string("gg_broadcast: ") + api_.last_error(engines_[k].e);
            return false;
        }
        owner_[value] = k;
        engines_[k].frozen = false;
        engines_[k].quiet_run = 0;
        engines_[k].queued = true;
        return true;
    }

    // a further engine over the same topology, at the same round
    bool add_engine(std::string& why) {
        gg_config c{};
        c.n_nodes = (uint64_t)V_;
        c.n_lanes = opt_.lanes;
        c.seed = opt_.seed;
        c.sync_base_ticks = 20;
        c.sync_jitter_ticks = 10;
        c.enable_sync = opt_.sync ? 1 : 0;
        c.batch_ticks = opt_.batch;
        c.device = opt_.device;
        c.world = 1;
        gg_engine* e = nullptr;
        int rc = api_.create(&c, &e);
        if (rc) {
            why = "gg_create failed: " + std::to_string(rc);
            return false;
        }
        rc = api_.topology(e, rp_.data(), col_.empty() ? nullptr : col_.data(), col_.size());
        // catch up with the current round: no values yet, so only the timers run
        if (rc == 0 && round_ > 0) rc = api_.step(e, (uint32_t)round_, nullptr);
        if (rc) {
            why = std::string("gg_topology/gg_step: ") + api_.last_error(e);
            api_.destroy(e);
            return false;
        }
        engines_.push_back({e, false, false});
        return true;
    }

    // Maelstrom error reply (code 13 = crash: the handler failed; the node keeps serving)
    bool error_reply(const std::string& from, const std::string& to, int64_t in_reply_to, const std::string& text) {
        std::string o = "{\"src\":";
        quote(o, from);
        o += ",\"dest\":";
        quote(o, to);
        o += ",\"body\":{\"code\":13,\"in_reply_to\":" + std::to_string(in_reply_to) + ",\"text\":";
        quote(o, text);
        o += ",\"type\":\"error\"}}\n";
        fwrite(o.data(), 1, o.size(), stdout);
        fflush(stdout);
        fprintf(stderr, "%s\n", text.c_str());
        return true;
    }

    bool fail(const std::string& what, int* status) {
        fprintf(stderr, "%s\n", what.c_str());
        *status = 1;
        return false;
    }

    bool reply(const std::string& from, const std::string& to, int64_t in_reply_to, const char* type,
               const std::string& extra, int*) {
        std::string o = "{\"src\":";
        quote(o, from);
        o += ",\"dest\":";
        quote(o, to);
        // the pinned maelstrom library's Reply re-marshals the body as a Go map,
        // so body keys come out in alphabetical order: in_reply_to, messages, type
        o += ",\"body\":{\"in_reply_to\":" + std::to_string(in_reply_to) + extra + ",\"type\":\"";
        o += type;
        o += "\"}}\n";
        fwrite(o.data(), 1, o.size(), stdout);
        fflush(stdout);
        if (opt_.log) fprintf(stderr, "Sent %s", o.c_str());
        return true;
    }

    // the engine for V nodes with the map's rows (a node without a row: no
    // neighbours, broadcast.go:41-42); `top` may be NUL (no topology yet)
    bool build(const Json& top, int* status) {
        int64_t V = n_nodes_;
        std::vector<std::vector<int32_t>> rows;
        if (top.kind == Json::OBJ) {
            for (const auto& kv : top.obj) {
                const int64_t u = node_index(kv.first);
                if (u < 0) return fail("topology key is not a node: " + kv.first, status);
                V = std::max(V, u + 1);
                for (const auto& x : kv.second.arr) V = std::max(V, node_index(x.str) + 1);
            }
        }
        if (V <= 0) return fail("node count unknown (no init, no topology)", status);
        rows.assign((size_t)V, {});
        if (top.kind == Json::OBJ) {
            for (const auto& kv : top.obj) {
                auto& r = rows[(size_t)node_index(kv.first)];
                for (const auto& x : kv.second.arr) {
                    const int64_t w = node_index(x.str);
                    if (w < 0) return fail("topology neighbour is not a node: " + x.str, status);
                    r.push_back((int32_t)w);
                }
            }
        }
        rp_.assign((size_t)V + 1, 0);
        col_.clear();
        for (int64_t v = 0; v < V; ++v) {
            auto& r = rows[(size_t)v];
            std::sort(r.begin(), r.end());
            r.erase(std::unique(r.begin(), r.end()), r.end());
            col_.insert(col_.end(), r.begin(), r.end());
            rp_[(size_t)v + 1] = (int64_t)col_.size();
        }
        sym_ = true;  // u lists w iff w lists u (an older engine may then freeze)
        for (int64_t u = 0; u < V && sym_; ++u)
            for (int32_t w : rows[(size_t)u])
                if (!std::binary_search(rows[(size_t)w].begin(), rows[(size_t)w].end(), (int32_t)u)) {
                    sym_ = false;
                    break;
                }
        V_ = V;
        std::string why;
        if (!add_engine(why)) return fail(why, status);
        return true;
    }

    Options opt_;
    Api& api_;
    std::vector<Slot> engines_;
    int64_t round_ = 0;  // rounds run so far (frozen engines lag behind it)
    std::unordered_map<int64_t, size_t> owner_;  // value -> engine
    std::vector<int64_t> rp_;
    std::vector<int32_t> col_;
    bool sym_ = true;
    bool windows_ = false;  // partition windows installed (none today: see can_freeze)
    int64_t V_ = 0;
    int64_t n_nodes_ = 0;
    std::map<uint32_t, std::vector<int64_t>> pending_;
};

std::string self_dir() {
    char buf[4096];
    const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
    if (n <= 0) return ".";
    std::string s(buf, (size_t)n);
    const size_t k = s.rfind('/');
    return k == std::string::npos ? "." : s.substr(0, k);
}

int usage() {
    fprintf(stderr,
            "usage: maelstrom-broadcast-hip [--engine LIB.so] [--lanes W] [--seed S] [--no-sync]\n"
            "                               [--batch B (batched gossip: one message per neighbour every B ticks)]\n"
            "                               [--device D] [--tick-ms T (0: lockstep, tick messages)] [--log]\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    o.engine = self_dir() + "/libgossip_hip.so";
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        const char* v = nullptr;
        if (a == "--engine" && (v = next())) o.engine = v;
        else if (a == "--lanes" && (v = next())) o.lanes = (uint32_t)strtoul(v, nullptr, 10);
        else if (a == "--seed" && (v = next())) o.seed = strtoull(v, nullptr, 0);
        else if (a == "--device" && (v = next())) o.device = atoi(v);
        else if (a == "--tick-ms" && (v = next())) o.tick_ms = atoi(v);
        else if (a == "--no-sync") o.sync = false;
        else if (a == "--batch" && (v = next())) o.batch = (uint32_t)strtoul(v, nullptr, 10);
        else if (a == "--log") o.log = true;
        else return usage();
    }
    Api api;
    std::string err;
    if (!api.load(o.engine, err)) {
        fprintf(stderr, "cannot load the engine: %s\n", err.c_str());
        return 1;
    }
    Front f(o, api);
    int status = 0;
    std::string line;
    if (o.tick_ms <= 0) {  // lockstep: rounds advance on tick messages only
        while (std::getline(std::cin, line)) {
            if (line.empty()) continue;
            if (!f.handle(line, &status)) return status;
        }
        return status;
    }
    // wall clock: one round per tick_ms, input handled between rounds
    using clk = std::chrono::steady_clock;
    auto next_tick = clk::now() + std::chrono::milliseconds(o.tick_ms);
    std::string buf;
    char chunk[65536];
    for (;;) {
        const auto now = clk::now();
        if (now >= next_tick) {
            if (!f.run_rounds(1, &status)) return status;
            next_tick += std::chrono::milliseconds(o.tick_ms);
            continue;
        }
        const int wait = (int)std::chrono::duration_cast<std::chrono::milliseconds>(next_tick - now).count();
        pollfd pfd{0, POLLIN, 0};
        const int pr = poll(&pfd, 1, wait);
        if (pr <= 0) continue;
        const ssize_t n = read(0, chunk, sizeof(chunk));
        if (n <= 0) return status;  // EOF
        buf.append(chunk, (size_t)n);
        size_t pos;
        while ((pos = buf.find('\n')) != std::string::npos) {
            line = buf.substr(0, pos);
            buf.erase(0, pos + 1);
            if (!line.empty() && !f.handle(line, &status)) return status;
        }
    }
}
