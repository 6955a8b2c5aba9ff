// graph.pkl without building the graph in Python: the pickle stream of the
// networkx Graph that build_graph (build_graph.py:40-68) makes from the gene
// matches tables, written directly.
//
// build_graph inserts, per table in order, the table's s-nodes (ssample,
// sgene) in row order, then its q-nodes (qsample, qgene), then its edges
// (s-node, q-node) in row order. A networkx Graph pickles as its __dict__
// ({"graph", "_node", "_adj", "__networkx_cache__"}) rebuilt on a new Graph:
// _node maps each node (a (sample name, gene) tuple) to its attribute dict in
// insertion order; _adj maps each node, in the same order, to {neighbour:
// edge data dict} in edge insertion order, the data dict shared by both ends.
// This writer emits exactly that object graph (protocol 4; every node tuple
// and edge dict memoised once, like pickle.dump), so pickle.load returns a
// Graph equal to build_graph's, node, neighbour and edge order included.
// At C3 (1.6 M nodes, 24.8 M edges) that takes seconds instead of the minutes
// of per-edge Python inserts plus pickle.dump.
#include "../../include/rcgpu.h"

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

int rcg_fail(int code, const std::string &msg);

namespace {

struct NodeKey {
    int64_t gene;
    int32_t sample;
};

// open-addressing hash maps (linear probing), 2^k slots
struct NodeMap {
    std::vector<NodeKey> key;
    std::vector<uint32_t> val;   // node id + 1 (0 = empty)
    size_t mask = 0, n = 0;
    static uint64_t h(const NodeKey &k)
    {
        uint64_t x = (uint64_t)k.gene * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)k.sample << 17);
        x ^= x >> 29;
        return x * 0xBF58476D1CE4E5B9ull;
    }
    void grow()
    {
        std::vector<NodeKey> ok;
        std::vector<uint32_t> ov;
        ok.swap(key);
        ov.swap(val);
        const size_t cap = ok.empty() ? (1u << 16) : ok.size() * 2;
        key.assign(cap, NodeKey{0, 0});
        val.assign(cap, 0);
        mask = cap - 1;
        for (size_t i = 0; i < ok.size(); i++)
            if (ov[i]) put(ok[i], ov[i]);
    }
    void put(const NodeKey &k, uint32_t v)
    {
        size_t i = h(k) & mask;
        while (val[i]) i = (i + 1) & mask;
        key[i] = k;
        val[i] = v;
    }
    // id of k, inserting `next` when absent (returns whether it was new)
    uint32_t get_or_add(const NodeKey &k, uint32_t next, bool &added)
    {
        if ((n + 1) * 2 > key.size()) grow();
        size_t i = h(k) & mask;
        while (val[i]) {
            if (key[i].gene == k.gene && key[i].sample == k.sample) {
                added = false;
                return val[i] - 1;
            }
            i = (i + 1) & mask;
        }
        key[i] = k;
        val[i] = next + 1;
        n++;
        added = true;
        return next;
    }
};

struct EdgeMap {
    std::vector<uint64_t> key;   // (lo << 32 | hi) + 1 (0 = empty)
    size_t mask = 0, n = 0;
    void grow()
    {
        std::vector<uint64_t> ok;
        ok.swap(key);
        const size_t cap = ok.empty() ? (1u << 16) : ok.size() * 2;
        key.assign(cap, 0);
        mask = cap - 1;
        for (uint64_t k : ok)
            if (k) {
                size_t i = slot(k - 1);
                while (key[i]) i = (i + 1) & mask;
                key[i] = k;
            }
    }
    size_t slot(uint64_t k) const
    {
        uint64_t x = k * 0x9E3779B97F4A7C15ull;
        return (size_t)(x ^ (x >> 31)) & mask;
    }
    bool add(uint64_t k)   // true when new
    {
        if ((n + 1) * 2 > key.size()) grow();
        size_t i = slot(k);
        while (key[i]) {
            if (key[i] == k + 1) return false;
            i = (i + 1) & mask;
        }
        key[i] = k + 1;
        n++;
        return true;
    }
};

}  // namespace

struct rc_gpickle {
    NodeMap nodes;                                 // genes outside [0, DENSE)
    std::vector<std::vector<uint32_t>> dense;      // per sample: gene -> node id + 1
    static constexpr int64_t DENSE = 1 << 26;
    std::vector<NodeKey> node;                     // insertion order
    // an edge joins two samples' genes, so only tables of the same sample pair
    // can repeat it: one small edge set per (unordered) sample pair, not one
    // set of every edge (random probes into a 25 M-entry table at C3)
    std::map<std::pair<int32_t, int32_t>, EdgeMap> emap;
    std::vector<std::pair<uint32_t, uint32_t>> edge;   // insertion order
};

extern "C" {

int rc_graph_pickle_begin(rc_gpickle **g)
{
    if (!g) return rcg_fail(RC_E_ARG, "null handle");
    *g = new rc_gpickle();
    return RC_OK;
}

void rc_graph_pickle_free(rc_gpickle *g) { delete g; }

int rc_graph_pickle_add(rc_gpickle *g, int32_t ssample, int32_t qsample, const int64_t *sgene, const int64_t *qgene,
                        uint64_t n)
{
    if (!g || (n && (!sgene || !qgene))) return rcg_fail(RC_E_ARG, "null argument");
    std::vector<uint32_t> su(n), qu(n);
    auto node_id = [&](int32_t s, int64_t gene) {
        bool added = false;
        const NodeKey k{gene, s};
        if (s >= 0 && gene >= 0 && gene < rc_gpickle::DENSE) {
            if ((size_t)s >= g->dense.size()) g->dense.resize((size_t)s + 1);
            std::vector<uint32_t> &d = g->dense[s];
            if ((size_t)gene >= d.size()) d.resize(std::max<size_t>((size_t)gene + 1, d.size() * 2), 0);
            if (!d[gene]) {
                d[gene] = (uint32_t)g->node.size() + 1;
                g->node.push_back(k);
            }
            return d[gene] - 1;
        }
        const uint32_t id = g->nodes.get_or_add(k, (uint32_t)g->node.size(), added);
        if (added) g->node.push_back(k);
        return id;
    };
    for (uint64_t i = 0; i < n; i++) su[i] = node_id(ssample, sgene[i]);
    for (uint64_t i = 0; i < n; i++) qu[i] = node_id(qsample, qgene[i]);
    EdgeMap &em = g->emap[{std::min(ssample, qsample), std::max(ssample, qsample)}];
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t a = su[i], b = qu[i];
        const uint64_t k = a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a);
        if (em.add(k)) g->edge.push_back({a, b});
    }
    if (g->node.size() >= 0x7FFFFFFFull || g->edge.size() >= 0x7FFFFFFFull)
        return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    return RC_OK;
}

int rc_graph_pickle_write(rc_gpickle *g, const char *path, int32_t n_names, const char *const *names)
{
    if (!g || !path || (n_names && !names)) return rcg_fail(RC_E_ARG, "null argument");
    const size_t nn = g->node.size(), ne = g->edge.size();
    for (const NodeKey &k : g->node)
        if (k.sample < 0 || k.sample >= n_names) return rcg_fail(RC_E_ARG, "sample index out of range");
    // adjacency in edge insertion order (CSR)
    std::vector<uint64_t> off(nn + 1, 0);
    for (auto &e : g->edge) {
        off[e.first + 1]++;
        if (e.second != e.first) off[e.second + 1]++;
    }
    for (size_t i = 0; i < nn; i++) off[i + 1] += off[i];
    std::vector<uint32_t> nbr(off[nn]), eid(off[nn]);
    {
        std::vector<uint64_t> cur(off.begin(), off.end() - 1);
        for (size_t i = 0; i < ne; i++) {
            const uint32_t a = g->edge[i].first, b = g->edge[i].second;
            nbr[cur[a]] = b;
            eid[cur[a]++] = (uint32_t)i;
            if (a != b) {
                nbr[cur[b]] = a;
                eid[cur[b]++] = (uint32_t)i;
            }
        }
    }
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return rcg_fail(RC_E_IO, "cannot open " + tmp);
    // the stream is built in a 16 MiB block and written a block at a time
    // (per-opcode stdio calls, each taking the FILE lock, ran at ~38 MB/s)
    const size_t BLK = 1u << 24;
    std::vector<uint8_t> blk(BLK + 4096);
    uint8_t *w = blk.data();
    uint8_t *const wend = blk.data() + BLK;
    bool werr = false;
    auto flush = [&]() {
        const size_t n = (size_t)(w - blk.data());
        if (n && fwrite(blk.data(), 1, n, f) != n) werr = true;
        w = blk.data();
    };
    uint32_t memo = 0;
    auto put = [&](const void *p, size_t n) {
        if (n > 4096) {   // a long sample name
            flush();
            if (fwrite(p, 1, n, f) != n) werr = true;
            return;
        }
        std::memcpy(w, p, n);
        w += n;
        if (w >= wend) flush();
    };
    auto op = [&](uint8_t c) {
        *w++ = c;
        if (w >= wend) flush();
    };
    auto u32 = [&](uint32_t v) { put(&v, 4); };
    auto memoize = [&]() { op(0x94); return memo++; };
    auto get = [&](uint32_t m) { op('j'); u32(m); };   // LONG_BINGET
    auto sstr = [&](const char *s) {                      // SHORT_BINUNICODE (< 256 bytes)
        const size_t n = strlen(s);
        op(0x8c);
        op((uint8_t)n);
        put(s, n);
    };
    auto integer = [&](int64_t v) {
        if (v >= 0 && v < 256) {
            op('K');
            op((uint8_t)v);
        } else if (v >= 0 && v < 65536) {
            op('M');
            const uint16_t w = (uint16_t)v;
            put(&w, 2);
        } else if (v >= INT32_MIN && v <= INT32_MAX) {
            op('J');
            const int32_t w = (int32_t)v;
            put(&w, 4);
        } else {   // LONG1: 8-byte two's complement
            op(0x8a);
            op(8);
            put(&v, 8);
        }
    };
    const uint32_t BATCH = 1000;   // items per SETITEMS, as pickle does
    op(0x80);
    op(4);   // PROTO 4
    sstr("networkx.classes.graph");
    memoize();
    sstr("Graph");
    memoize();
    op(0x93);   // STACK_GLOBAL
    memoize();
    op(')');    // EMPTY_TUPLE
    op(0x81);   // NEWOBJ
    memoize();
    op('}');    // the state dict
    memoize();
    op('(');
    sstr("graph");
    memoize();
    op('}');
    memoize();
    // sample names, memoised once (BINUNICODE)
    std::vector<uint32_t> name_memo(n_names, 0xFFFFFFFFu);
    std::vector<uint32_t> node_memo(nn);
    sstr("_node");
    memoize();
    op('}');
    memoize();
    for (size_t i0 = 0; i0 < nn; i0 += BATCH) {
        op('(');
        for (size_t i = i0; i < nn && i < i0 + BATCH; i++) {
            const NodeKey &k = g->node[i];
            if (name_memo[k.sample] == 0xFFFFFFFFu) {
                const uint32_t len = (uint32_t)strlen(names[k.sample]);
                op('X');
                u32(len);
                put(names[k.sample], len);
                name_memo[k.sample] = memoize();
            } else {
                get(name_memo[k.sample]);
            }
            integer(k.gene);
            op(0x86);   // TUPLE2
            node_memo[i] = memoize();
            op('}');    // the node's attribute dict
            memoize();
        }
        op('u');        // SETITEMS
    }
    sstr("_adj");
    memoize();
    op('}');
    memoize();
    std::vector<uint32_t> edge_memo(ne, 0xFFFFFFFFu);
    for (size_t i0 = 0; i0 < nn; i0 += BATCH) {
        op('(');
        for (size_t i = i0; i < nn && i < i0 + BATCH; i++) {
            get(node_memo[i]);
            op('}');
            memoize();
            for (uint64_t j0 = off[i]; j0 < off[i + 1]; j0 += BATCH) {
                op('(');
                for (uint64_t j = j0; j < off[i + 1] && j < j0 + BATCH; j++) {
                    get(node_memo[nbr[j]]);
                    uint32_t &em = edge_memo[eid[j]];
                    if (em == 0xFFFFFFFFu) {
                        op('}');
                        em = memoize();
                    } else {
                        get(em);
                    }
                }
                op('u');
            }
        }
        op('u');
    }
    sstr("__networkx_cache__");
    memoize();
    op('}');
    memoize();
    op('u');    // SETITEMS of the state dict
    op('b');    // BUILD
    op('.');    // STOP
    flush();
    const bool bad = werr || ferror(f) != 0;
    if (fclose(f) != 0 || bad) {
        remove(tmp.c_str());
        return rcg_fail(RC_E_IO, "write failed: " + tmp);
    }
    if (rename(tmp.c_str(), path) != 0) return rcg_fail(RC_E_IO, std::string("cannot rename to ") + path);
    return RC_OK;
}

}  // extern "C"
