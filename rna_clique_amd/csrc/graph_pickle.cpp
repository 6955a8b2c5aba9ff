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
//
// Every phase runs on a pool of threads (r06; C5: 12.8 M nodes, 807 M edges,
// a 14 GB stream):
//  * nodes are numbered per sample -- a node belongs to one sample, so each
//    sample walks the tables that hold it, in order, to find its nodes' first
//    occurrences, and the (table, side) runs of first occurrences place them
//    (no global atomics, no global sort);
//  * edges are deduplicated per sample pair (only tables of the same pair can
//    repeat an edge) -- or not at all when the caller's records are unique
//    (the engine's edge records are one per edge already);
//  * adjacency lists (CSR) in edge insertion order from node-range buckets;
//  * memo numbers and every stream piece's exact byte size by prefix sums, so
//    each piece is written straight into a shared mapping of the file at its
//    offset (page-cache writes from every thread; pwrite on one file
//    serialises on the inode lock).
#include "../../include/rcgpu.h"
#include "graph_pickle.h"

#include <cstdint>
#include <cstdio>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <map>
#include <new>
#include <memory>
#include <string>
#include <vector>

int rcg_fail(int code, const std::string &msg);

static constexpr size_t RAW_MAP_MIN = 32ull << 20;

void *raw_alloc(size_t bytes)
{
    if (bytes < RAW_MAP_MIN) {
        void *p = std::malloc(bytes);
        if (!p) throw std::bad_alloc();
        return p;
    }
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    madvise(p, bytes, MADV_HUGEPAGE);
    return p;
}

void raw_free(void *p, size_t bytes)
{
    if (bytes < RAW_MAP_MIN) std::free(p);
    else munmap(p, bytes);
}

namespace {

using NodeKey = GraphNodeKey;

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
    // the tables as given (their gene arrays), in call order
    struct Tab {
        int32_t ss, qs;   // s- and q-sample
        uint64_t n;
        Raw<int64_t> sg, qg;
    };
    uint64_t rows = 0;
    std::vector<Tab> tabs;
};

namespace {

// worker threads for the write: the CPUs this process may use, at most 16
// (the GPU box's quota)
int pool_size()
{
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

// run f(i) for i in [0, n) on the pool, dynamically (an atomic counter)
template <class F>
void parallel_for(size_t n, F f)
{
    const int T = (int)std::min<size_t>((size_t)pool_size(), std::max<size_t>(n, 1));
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

// the pickle opcodes this writer emits, at a write pointer (into a buffer of
// its own, or into the file mapping at the piece's offset)
struct Out {
    Raw<char> buf;
    char *w = nullptr;
    Out() = default;
    explicit Out(size_t cap) : buf(cap), w(buf.data()) {}
    size_t size() const { return (size_t)(w - buf.data()); }
    void op(uint8_t c) { *w++ = (char)c; }
    void put(const void *p, size_t n)
    {
        std::memcpy(w, p, n);
        w += n;
    }
    void u32(uint32_t v) { put(&v, 4); }
    void memoize() { op(0x94); }
    void get(uint32_t m)   // LONG_BINGET
    {
        op('j');
        u32(m);
    }
    void sstr(const char *s)   // SHORT_BINUNICODE (< 256 bytes)
    {
        const size_t n = strlen(s);
        op(0x8c);
        op((uint8_t)n);
        put(s, n);
    }
    void integer(int64_t v)
    {
        if (v >= 0 && v < 256) {
            op('K');
            op((uint8_t)v);
        } else if (v >= 0 && v < 65536) {
            op('M');
            const uint16_t x = (uint16_t)v;
            put(&x, 2);
        } else if (v >= INT32_MIN && v <= INT32_MAX) {
            op('J');
            const int32_t x = (int32_t)v;
            put(&x, 4);
        } else {   // LONG1: 8-byte two's complement
            op(0x8a);
            op(8);
            put(&v, 8);
        }
    }
};

// bytes of Out::integer(v)
inline size_t int_bytes(int64_t v)
{
    if (v >= 0 && v < 256) return 2;
    if (v >= 0 && v < 65536) return 3;
    if (v >= INT32_MIN && v <= INT32_MAX) return 5;
    return 10;
}

}  // namespace

namespace {

// Node ids in build_graph's insertion order (per table its s-nodes, then its
// q-nodes, tables in call order): a node's id is the rank of its first
// occurrence. U and V are rewritten from slots to ids.
void number_nodes(GraphSlots &G)
{
    const size_t nt = G.tabs.size();
    const int32_t ns = G.ns;
    // the (table, side) lists of every sample, in build_graph's order
    std::vector<std::vector<uint64_t>> stabs((size_t)ns);
    for (size_t t = 0; t < nt; t++) {
        if (!G.tabs[t].n) continue;
        stabs[G.tabs[t].ss].push_back((uint64_t)t << 1);
        stabs[G.tabs[t].qs].push_back(((uint64_t)t << 1) | 1u);
    }
    // per sample: its nodes' first occurrences (ts << 32 | row), sorted
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> occ((size_t)ns);
    std::vector<uint64_t> run((size_t)2 * nt + 1, 0);   // new nodes per (table, side)
    parallel_for((size_t)ns, [&](size_t s) {
        const uint64_t b0 = G.base[s], cnt = G.base[s + 1] - b0;
        if (stabs[s].empty() || !cnt) return;
        std::vector<uint64_t> first(cnt, ~0ull);
        uint64_t nf = 0;
        for (uint64_t ts : stabs[s]) {
            const GraphSlots::Tab &T = G.tabs[ts >> 1];
            const uint32_t *A = ((ts & 1) ? G.V.data() : G.U.data()) + T.off;
            for (uint64_t i = 0; i < T.n; i++) {
                uint64_t &f = first[A[i] - b0];
                if (f == ~0ull) {
                    f = (ts << 32) | i;
                    nf++;
                }
            }
            if (nf == cnt) break;   // every slot of the sample seen
        }
        std::vector<std::pair<uint64_t, uint32_t>> &o = occ[s];
        o.reserve(nf);
        for (uint64_t k = 0; k < cnt; k++)
            if (first[k] != ~0ull) o.push_back({first[k], (uint32_t)k});
        std::sort(o.begin(), o.end());
        for (const auto &x : o) run[(x.first >> 32) + 1]++;   // (every ts belongs to this sample alone)
    });
    for (size_t k = 0; k < 2 * nt; k++) run[k + 1] += run[k];
    const uint64_t nn = run[2 * nt];
    G.node.resize(nn);
    Raw<uint32_t> id(G.base[ns]);
    parallel_for((size_t)ns, [&](size_t s) {
        const uint64_t b0 = G.base[s];
        const auto &o = occ[s];
        uint64_t cur = ~0ull, at = 0;
        for (const auto &x : o) {
            const uint64_t ts = x.first >> 32;
            if (ts != cur) {
                cur = ts;
                at = run[ts];
            }
            const uint64_t slot = b0 + x.second;
            id[slot] = (uint32_t)at;
            G.node[at] = NodeKey{G.slot_gene ? (int64_t)G.slot_gene[slot] : (int64_t)x.second, (int32_t)s};
            at++;
        }
    });
    occ.clear();
    parallel_for(nt, [&](size_t t) {
        const GraphSlots::Tab &T = G.tabs[t];
        for (uint64_t i = T.off; i < T.off + T.n; i++) {
            G.U[i] = id[G.U[i]];
            G.V[i] = id[G.V[i]];
        }
    });
    G.ids = true;
}

// The API's tables (int64 genes) as slots: dense gene ranges per sample when
// every gene is in [0, 2^26) and the ranges are not much larger than the rows;
// otherwise node ids by the sequential walk with a hash map
void tables_to_slots(rc_gpickle *g, GraphSlots &G)
{
    const size_t nt = g->tabs.size();
    int32_t ns = 0;
    bool dense = true;
    for (auto &T : g->tabs) {
        dense = dense && T.ss >= 0 && T.qs >= 0;
        ns = std::max(ns, std::max(T.ss, T.qs) + 1);
    }
    G.ns = ns;
    G.tabs.resize(nt);
    uint64_t off = 0;
    for (size_t t = 0; t < nt; t++) {
        G.tabs[t] = GraphSlots::Tab{g->tabs[t].ss, g->tabs[t].qs, off, g->tabs[t].n};
        off += g->tabs[t].n;
    }
    G.rows = off;
    G.U = Raw<uint32_t>(off);
    G.V = Raw<uint32_t>(off);
    constexpr int64_t DENSE = 1 << 26;
    std::vector<int64_t> gmax((size_t)ns, -1);
    if (dense) {
        std::vector<int64_t> tmin(nt, 0), tsmax(nt, -1), tqmax(nt, -1);
        parallel_for(nt, [&](size_t t) {
            const rc_gpickle::Tab &T = g->tabs[t];
            int64_t mn = 0, sx = -1, qx = -1;
            for (uint64_t i = 0; i < T.n; i++) {
                mn = std::min(mn, std::min(T.sg[i], T.qg[i]));
                sx = std::max(sx, T.sg[i]);
                qx = std::max(qx, T.qg[i]);
            }
            tmin[t] = mn;
            tsmax[t] = sx;
            tqmax[t] = qx;
        });
        for (size_t t = 0; t < nt; t++) {
            dense = dense && tmin[t] >= 0;
            gmax[g->tabs[t].ss] = std::max(gmax[g->tabs[t].ss], tsmax[t]);
            gmax[g->tabs[t].qs] = std::max(gmax[g->tabs[t].qs], tqmax[t]);
        }
    }
    G.base.assign((size_t)ns + 1, 0);
    for (int32_t k = 0; k < ns; k++) {
        dense = dense && gmax[k] < DENSE;
        G.base[k + 1] = G.base[k] + (uint64_t)(gmax[k] + 1);
    }
    dense = dense && G.base[ns] <= 4 * off + (1u << 24) && G.base[ns] < 0xFFFFFFFFull;
    if (dense) {
        parallel_for(nt, [&](size_t t) {
            const rc_gpickle::Tab &T = g->tabs[t];
            const uint64_t o = G.tabs[t].off, bs = G.base[T.ss], bq = G.base[T.qs];
            for (uint64_t i = 0; i < T.n; i++) {
                G.U[o + i] = (uint32_t)(bs + (uint64_t)T.sg[i]);
                G.V[o + i] = (uint32_t)(bq + (uint64_t)T.qg[i]);
            }
        });
        return;
    }
    NodeMap nodes;
    for (size_t t = 0; t < nt; t++) {
        const rc_gpickle::Tab &T = g->tabs[t];
        auto node_id = [&](int32_t s, int64_t gene) {
            bool added = false;
            const NodeKey k{gene, s};
            const uint32_t id = nodes.get_or_add(k, (uint32_t)G.node.size(), added);
            if (added) G.node.push_back(k);
            return id;
        };
        const uint64_t o = G.tabs[t].off;
        for (uint64_t i = 0; i < T.n; i++) G.U[o + i] = node_id(T.ss, T.sg[i]);
        for (uint64_t i = 0; i < T.n; i++) G.V[o + i] = node_id(T.qs, T.qg[i]);
    }
    G.ids = true;
}

}  // namespace

// the whole write from slot form (engine.hip hands its device-sorted edge
// records in this form; rc_graph_pickle_write its tables)
int graph_pickle_write_slots(GraphSlots &G, const char *path, int32_t n_names, const char *const *names)
{
    if (!path || (n_names && !names)) return rcg_fail(RC_E_ARG, "null argument");
    const bool tmg = getenv("RC_OUT_TIMING") && atoi(getenv("RC_OUT_TIMING"));
    auto clk = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!tmg) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "graph.pkl %s %.3f s\n", what, std::chrono::duration<double>(t - clk).count());
        clk = t;
    };
    if (G.tabs.size() >= 0x7FFFFFFFull || G.rows >= 0xFFFFFFFFull)
        return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    for (const auto &T : G.tabs)
        if (T.n && (T.ss < 0 || T.qs < 0 || T.ss >= n_names || T.qs >= n_names))
            return rcg_fail(RC_E_ARG, "sample index out of range");
    if (!G.ids) number_nodes(G);
    lap("nodes");
    if (G.node.size() >= 0x7FFFFFFFull) return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    const size_t nn = G.node.size(), nt = G.tabs.size();
    for (const NodeKey &k : G.node)
        if (k.sample < 0 || k.sample >= n_names) return rcg_fail(RC_E_ARG, "sample index out of range");
    // 1. the edges: first occurrence of each (s-node, q-node) pair, per
    // sample-pair group of tables (in call order) on its own thread -- unless
    // the caller's rows are unique edges already (then the rows are the edges)
    Raw<uint32_t> EU, EV;
    const uint32_t *eu = G.U.data(), *ev = G.V.data();
    size_t ne = G.rows;
    if (!G.unique) {
        Raw<uint8_t> keep(G.rows);
        std::map<std::pair<int32_t, int32_t>, std::vector<uint32_t>> groups;
        for (size_t t = 0; t < nt; t++)
            groups[{std::min(G.tabs[t].ss, G.tabs[t].qs), std::max(G.tabs[t].ss, G.tabs[t].qs)}].push_back((uint32_t)t);
        std::vector<const std::vector<uint32_t> *> gl;
        for (auto &kv : groups) gl.push_back(&kv.second);
        parallel_for(gl.size(), [&](size_t k) {
            uint64_t rows = 0;
            for (uint32_t t : *gl[k]) rows += G.tabs[t].n;
            EdgeMap em;
            while (em.key.size() < 2 * rows + 2) em.grow();
            for (uint32_t t : *gl[k]) {
                const GraphSlots::Tab &T = G.tabs[t];
                for (uint64_t i = T.off; i < T.off + T.n; i++) {
                    const uint32_t a = G.U[i], b = G.V[i];
                    keep[i] = em.add(a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a)) ? 1 : 0;
                }
            }
        });
        // edges in insertion order: tables in call order, rows in order
        std::vector<uint64_t> tcount(nt + 1, 0);
        parallel_for(nt, [&](size_t t) {
            uint64_t c = 0;
            for (uint64_t i = G.tabs[t].off; i < G.tabs[t].off + G.tabs[t].n; i++) c += keep[i];
            tcount[t + 1] = c;
        });
        for (size_t t = 0; t < nt; t++) tcount[t + 1] += tcount[t];
        ne = tcount[nt];
        EU = Raw<uint32_t>(ne);
        EV = Raw<uint32_t>(ne);
        parallel_for(nt, [&](size_t t) {
            uint64_t w = tcount[t];
            for (uint64_t i = G.tabs[t].off; i < G.tabs[t].off + G.tabs[t].n; i++)
                if (keep[i]) {
                    EU[w] = G.U[i];
                    EV[w++] = G.V[i];
                }
        });
        eu = EU.data();
        ev = EV.data();
        G.U = Raw<uint32_t>();
        G.V = Raw<uint32_t>();
    }
    lap("edges");
    // 2. adjacency in edge insertion order (CSR), built in parallel: the
    // (node, neighbour, edge) entries are stably partitioned into node-range
    // buckets (per-thread counts over chunks of edges, then a scatter in
    // chunk order), and each bucket's nodes get their lists on one thread --
    // random writes stay inside a bucket instead of spanning the whole graph
    std::vector<uint64_t> off(nn + 1, 0);
    Raw<uint32_t> nbr, eid;
    {
        const int NB = 256;
        const uint64_t span = std::max<uint64_t>(1, (nn + NB - 1) / NB);
        const size_t ECH = 1u << 20;   // edges per chunk
        const size_t nec = (ne + ECH - 1) / ECH;
        std::vector<uint64_t> cnt((nec + 1) * NB, 0);   // [chunk][bucket]
        parallel_for(nec, [&](size_t c) {
            uint64_t *h = &cnt[c * NB];
            for (size_t i = c * ECH; i < std::min(ne, (c + 1) * ECH); i++) {
                h[eu[i] / span]++;
                if (ev[i] != eu[i]) h[ev[i] / span]++;
            }
        });
        // exclusive prefix in (bucket, chunk) order: bucket-major, chunks in order
        std::vector<uint64_t> bstart(NB + 1, 0);
        {
            uint64_t run = 0;
            for (int bk = 0; bk < NB; bk++) {
                bstart[bk] = run;
                for (size_t c = 0; c < nec; c++) {
                    const uint64_t v = cnt[c * NB + bk];
                    cnt[c * NB + bk] = run;
                    run += v;
                }
            }
            bstart[NB] = run;
        }
        struct Ent {
            uint32_t u, v, e;
        };
        Raw<Ent> ent(bstart[NB]);
        parallel_for(nec, [&](size_t c) {
            uint64_t *h = &cnt[c * NB];
            for (size_t i = c * ECH; i < std::min(ne, (c + 1) * ECH); i++) {
                const uint32_t a = eu[i], b2 = ev[i];
                ent[h[a / span]++] = Ent{a, b2, (uint32_t)i};
                if (a != b2) ent[h[b2 / span]++] = Ent{b2, a, (uint32_t)i};
            }
        });
        lap("csr scatter");
        // per bucket: degrees, then its nodes' offsets (global, once the
        // buckets' totals are known: bstart), then the lists in entry order
        parallel_for(NB, [&](size_t bk) {
            for (uint64_t k = bstart[bk]; k < bstart[bk + 1]; k++) off[ent[k].u + 1]++;
        });
        for (size_t i = 0; i < nn; i++) off[i + 1] += off[i];
        nbr = Raw<uint32_t>(off[nn]);
        eid = Raw<uint32_t>(off[nn]);
        parallel_for(NB, [&](size_t bk) {
            const uint64_t lo = std::min<uint64_t>(nn, bk * span), hi = std::min<uint64_t>(nn, (bk + 1) * span);
            if (lo >= hi) return;
            std::vector<uint64_t> cur(off.begin() + lo, off.begin() + hi);
            for (uint64_t k = bstart[bk]; k < bstart[bk + 1]; k++) {
                const Ent &x = ent[k];
                const uint64_t w = cur[x.u - lo]++;
                nbr[w] = x.v;
                eid[w] = x.e;
            }
        });
    }
    EU = Raw<uint32_t>();
    EV = Raw<uint32_t>();
    G.U = Raw<uint32_t>();
    G.V = Raw<uint32_t>();
    lap("csr");
    // 3. memo numbers, as a sequential pickle.dump assigns them: 9 memos
    // before the first node; per node entry its sample name (first time the
    // sample appears), its tuple and its attribute dict; then "_adj" and its
    // dict; per adjacency entry the node's dict and the data dict of every
    // edge seen there first (at its lower-numbered end: node ids are stream
    // order; a self-loop's dict is made at its only node)
    const uint32_t BATCH = 1000;   // items per SETITEMS, as pickle does
    std::vector<uint32_t> name_memo(n_names, 0xFFFFFFFFu), node_memo(nn);
    std::vector<uint8_t> name_here(nn, 0);
    uint64_t memo = 9;
    for (size_t i = 0; i < nn; i++) {
        const int32_t s = G.node[i].sample;
        if (name_memo[s] == 0xFFFFFFFFu) {
            name_memo[s] = (uint32_t)memo++;
            name_here[i] = 1;
        }
        node_memo[i] = (uint32_t)memo;
        memo += 2;
    }
    memo += 2;   // "_adj", its dict
    std::vector<uint64_t> adj_memo(nn + 1);
    std::vector<uint32_t> nnew(nn, 0);   // new edge dicts per node (neighbour ids above the node, or itself)
    parallel_for((nn + 65535) / 65536, [&](size_t c) {
        for (size_t i = c * 65536; i < std::min(nn, (c + 1) * 65536); i++) {
            uint32_t k = 0;
            for (uint64_t j = off[i]; j < off[i + 1]; j++) k += nbr[j] >= i;
            nnew[i] = k;
        }
    });
    for (size_t i = 0; i < nn; i++) {
        adj_memo[i] = memo;
        memo += 1 + nnew[i];
    }
    adj_memo[nn] = memo;
    if (memo >= 0xFFFFFFFFull) return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    Raw<uint32_t> edge_memo(ne);
    parallel_for((nn + 65535) / 65536, [&](size_t c) {
        for (size_t i = c * 65536; i < std::min(nn, (c + 1) * 65536); i++) {
            uint64_t m = adj_memo[i] + 1;
            for (uint64_t j = off[i]; j < off[i + 1]; j++)
                if (nbr[j] >= i) edge_memo[eid[j]] = (uint32_t)m++;
        }
    });
    lap("memo");
    // 4. the stream: head, node entries and adjacency entries in chunks of
    // whole SETITEMS batches, tail. Every piece's exact size first (prefix
    // sums), then each chunk is written on the pool straight to its offset
    Out head(4096);
    head.op(0x80);
    head.op(4);   // PROTO 4
    head.sstr("networkx.classes.graph");
    head.memoize();
    head.sstr("Graph");
    head.memoize();
    head.op(0x93);   // STACK_GLOBAL
    head.memoize();
    head.op(')');    // EMPTY_TUPLE
    head.op(0x81);   // NEWOBJ
    head.memoize();
    head.op('}');    // the state dict
    head.memoize();
    head.op('(');
    head.sstr("graph");
    head.memoize();
    head.op('}');
    head.memoize();
    head.sstr("_node");
    head.memoize();
    head.op('}');
    head.memoize();
    Out mid(256), tail(256);
    mid.sstr("_adj");
    mid.memoize();
    mid.op('}');
    mid.memoize();
    tail.sstr("__networkx_cache__");
    tail.memoize();
    tail.op('}');
    tail.memoize();
    tail.op('u');    // SETITEMS of the state dict
    tail.op('b');    // BUILD
    tail.op('.');    // STOP
    const size_t CH = 64 * BATCH;   // nodes per chunk
    const size_t nch = (nn + CH - 1) / CH;
    std::vector<size_t> name_len(n_names);
    for (int32_t k = 0; k < n_names; k++) name_len[k] = strlen(names[k]);
    // piece k: 0 head, 1..nch node chunks, nch + 1 mid, nch + 2.. adjacency
    // chunks, 2 nch + 2 tail
    const size_t np = 2 * nch + 3;
    std::vector<uint64_t> at(np + 1, 0);
    at[1] = head.size();
    at[nch + 2] = mid.size();
    at[np] = tail.size();
    parallel_for(2 * nch, [&](size_t x) {
        const size_t c = x % nch, i0 = c * CH, i1 = std::min(nn, (c + 1) * CH);
        uint64_t b = 2 * ((i1 - i0 + BATCH - 1) / BATCH);   // '(' 'u' per batch
        if (x < nch) {
            // name ('X' + length + bytes + memo) or its get, the gene,
            // TUPLE2 + memo + '}' + memo
            for (size_t i = i0; i < i1; i++)
                b += (name_here[i] ? 6 + name_len[G.node[i].sample] : 5) + int_bytes(G.node[i].gene) + 4;
            at[c + 2] = b;
        } else {
            // get + '}' + memo; per neighbour its get and the dict ('}' +
            // memo) or the dict's get; '(' 'u' per neighbour batch
            for (size_t i = i0; i < i1; i++) {
                const uint64_t d = off[i + 1] - off[i];
                b += 7 + 5 * d + 2 * (uint64_t)nnew[i] + 5 * (d - nnew[i]) + 2 * ((d + BATCH - 1) / BATCH);
            }
            at[nch + c + 3] = b;
        }
    });
    for (size_t k = 0; k < np; k++) at[k + 1] += at[k];
    const uint64_t total = at[np];
    const std::string tmp = std::string(path) + ".tmp";
    const int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return rcg_fail(RC_E_IO, "cannot open " + tmp);
    std::atomic<bool> werr{ftruncate(fd, (off_t)total) != 0};
    // RC_PICKLE_MMAP=1: every thread writes into a shared mapping of the file
    // (no inode lock; but a page fault per 4 KB of file: 6.1 s for C5's 14 GB
    // on the GPU box vs ~1.5 s of pwrite). Default: each piece is built in
    // its thread's reused buffer and pwritten at its offset.
    char *map = nullptr;
    const char *mv = getenv("RC_PICKLE_MMAP");
    if (mv && atoi(mv) && !werr && total) {
        void *m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) map = static_cast<char *>(m);
    }
    std::atomic<bool> bad_size{false};
    auto emit = [&](size_t k, auto &&body) {
        const uint64_t n = at[k + 1] - at[k];
        static thread_local Raw<char> tbuf;
        Out o;
        if (map) {
            o.w = map + at[k];
        } else {
            if (tbuf.n < n + 16) tbuf = Raw<char>(std::max<size_t>(n + 16, (size_t)1 << 20));
            o.w = tbuf.data();
        }
        char *const start = o.w;
        body(o);
        if ((uint64_t)(o.w - start) != n) {
            bad_size = true;
            return;
        }
        if (!map) {
            uint64_t done = 0;
            while (done < n && !werr) {
                const ssize_t r = pwrite(fd, start + done, std::min<uint64_t>(n - done, 1u << 30), (off_t)(at[k] + done));
                if (r <= 0) werr = true;
                else done += (uint64_t)r;
            }
        }
    };
    if (!werr) {
        auto small = [&](const Out &src) { return [&src](Out &o) { o.put(src.buf.data(), src.size()); }; };
        emit(0, small(head));
        emit(nch + 1, small(mid));
        emit(np - 1, small(tail));
        parallel_for(2 * nch, [&](size_t x) {
            const size_t c = x % nch, i1 = std::min(nn, (c + 1) * CH);
            if (x < nch) {
                emit(c + 1, [&](Out &o) {
                    for (size_t i0 = c * CH; i0 < i1; i0 += BATCH) {
                        o.op('(');
                        for (size_t i = i0; i < i1 && i < i0 + BATCH; i++) {
                            const NodeKey &k = G.node[i];
                            if (name_here[i]) {
                                const uint32_t len = (uint32_t)name_len[k.sample];
                                o.op('X');
                                o.u32(len);
                                o.put(names[k.sample], len);
                                o.memoize();
                            } else {
                                o.get(name_memo[k.sample]);
                            }
                            o.integer(k.gene);
                            o.op(0x86);   // TUPLE2
                            o.memoize();
                            o.op('}');    // the node's attribute dict
                            o.memoize();
                        }
                        o.op('u');        // SETITEMS
                    }
                });
            } else {
                emit(nch + c + 2, [&](Out &o) {
                    for (size_t i0 = c * CH; i0 < i1; i0 += BATCH) {
                        o.op('(');
                        for (size_t i = i0; i < i1 && i < i0 + BATCH; i++) {
                            o.get(node_memo[i]);
                            o.op('}');
                            o.memoize();
                            for (uint64_t j0 = off[i]; j0 < off[i + 1]; j0 += BATCH) {
                                o.op('(');
                                for (uint64_t j = j0; j < off[i + 1] && j < j0 + BATCH; j++) {
                                    o.get(node_memo[nbr[j]]);
                                    if (nbr[j] >= i) {   // the edge's dict, first seen here
                                        o.op('}');
                                        o.memoize();
                                    } else {
                                        o.get(edge_memo[eid[j]]);
                                    }
                                }
                                o.op('u');
                            }
                        }
                        o.op('u');
                    }
                });
            }
        });
    }
    lap("stream");
    if (map) munmap(map, total);
    if (close(fd) != 0 || werr || bad_size) {
        remove(tmp.c_str());
        return bad_size ? rcg_fail(RC_E_STATE, "graph.pkl: stream size model mismatch")
                        : rcg_fail(RC_E_IO, "write failed: " + tmp);
    }
    if (rename(tmp.c_str(), path) != 0) return rcg_fail(RC_E_IO, std::string("cannot rename to ") + path);
    lap("file");
    // the big arrays are unmapped on a thread of their own (C5: ~16 GB,
    // 1.6 s of munmap the caller need not wait for)
    struct Hold {
        Raw<uint32_t> a, b, c;
    };
    auto *h = new Hold{std::move(nbr), std::move(eid), std::move(edge_memo)};
    std::thread([h]() { delete h; }).detach();
    return RC_OK;
}

extern "C" {

int rc_graph_pickle_begin(rc_gpickle **g)
{
    if (!g) return rcg_fail(RC_E_ARG, "null handle");
    *g = new rc_gpickle();
    return RC_OK;
}

void rc_graph_pickle_free(rc_gpickle *g) { delete g; }

// a table's gene arrays, to be filled by the caller (rc_write_outputs'
// graph thread writes them in place); see rc_graph_pickle_add
int graph_pickle_table(rc_gpickle *g, int32_t ssample, int32_t qsample, uint64_t n, int64_t **sgene, int64_t **qgene)
{
    rc_gpickle::Tab T;
    T.ss = ssample;
    T.qs = qsample;
    T.n = n;
    T.sg = Raw<int64_t>(n);
    T.qg = Raw<int64_t>(n);
    *sgene = T.sg.data();
    *qgene = T.qg.data();
    g->tabs.push_back(std::move(T));
    g->rows += n;
    if (g->tabs.size() >= 0x7FFFFFFFull || g->rows >= 0xFFFFFFFFull)
        return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    return RC_OK;
}

int rc_graph_pickle_add(rc_gpickle *g, int32_t ssample, int32_t qsample, const int64_t *sgene, const int64_t *qgene,
                        uint64_t n)
{
    if (!g || (n && (!sgene || !qgene))) return rcg_fail(RC_E_ARG, "null argument");
    int64_t *sg = nullptr, *qg = nullptr;
    const int rc = graph_pickle_table(g, ssample, qsample, n, &sg, &qg);
    if (n) {
        std::memcpy(sg, sgene, n * 8);
        std::memcpy(qg, qgene, n * 8);
    }
    return rc;
}

int rc_graph_pickle_write(rc_gpickle *g, const char *path, int32_t n_names, const char *const *names)
{
    if (!g || !path || (n_names && !names)) return rcg_fail(RC_E_ARG, "null argument");
    for (const auto &T : g->tabs)
        if (T.n && (T.ss < 0 || T.qs < 0 || T.ss >= n_names || T.qs >= n_names))
            return rcg_fail(RC_E_ARG, "sample index out of range");
    const auto t0 = std::chrono::steady_clock::now();
    GraphSlots G;
    tables_to_slots(g, G);
    g->tabs.clear();
    if (getenv("RC_OUT_TIMING") && atoi(getenv("RC_OUT_TIMING")))
        fprintf(stderr, "graph.pkl tables to slots %.3f s\n",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return graph_pickle_write_slots(G, path, n_names, names);
}

}  // extern "C"
