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
#include <fcntl.h>
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <map>
#include <memory>
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

// an array of trivially constructible T left uninitialised (new T[n]): its
// pages are first touched by the threads that fill it, not zeroed up front on
// one thread (hundreds of MB at C3, tens of GB at C5)
template <class T>
struct Raw {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    Raw() = default;
    explicit Raw(size_t k) : p(k ? new T[k] : nullptr), n(k) {}
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
    T *data() { return p.get(); }
};

struct rc_gpickle {
    NodeMap nodes;                                 // genes outside [0, DENSE) (sequential numbering)
    std::vector<std::vector<uint32_t>> dense;      // per sample: gene -> node id + 1 (sequential numbering)
    static constexpr int64_t DENSE = 1 << 26;
    std::vector<NodeKey> node;                     // insertion order
    // the tables as given (their gene arrays), in call order; node ids
    // (first occurrences in build_graph's order) and edges (first occurrences
    // of each node pair) are found at write time, in parallel: an edge joins
    // two samples' genes, so only tables of the same sample pair can repeat it
    struct Tab {
        int32_t ss, qs;   // s- and q-sample
        int32_t lo, hi;   // the sample pair (unordered)
        uint64_t off, n;  // its rows (a running row count over the tables)
        Raw<int64_t> sg, qg;
        Raw<uint32_t> su, qu;
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

// the pickle opcodes this writer emits, into a buffer sized up front (an
// upper bound of what the writer puts there: no growth, no zero fill)
struct Out {
    Raw<char> buf;
    char *w = nullptr;
    Out() = default;
    explicit Out(size_t cap) : buf(cap), w(buf.data()) {}
    size_t size() const { return (size_t)(w - buf.p.get()); }
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

}  // namespace

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
    T.lo = std::min(ssample, qsample);
    T.hi = std::max(ssample, qsample);
    T.off = g->rows;
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

// Node ids in build_graph's insertion order (per table its s-nodes, then its
// q-nodes, tables in call order): a node's id is the rank of its first
// occurrence. Dense genes (every gene in [0, DENSE) and the per-sample gene
// ranges not much larger than the rows): the first occurrence of each
// (sample, gene) slot by an atomic min over all rows in parallel, the slots
// ordered by it. Otherwise the sequential walk with a hash map.
static void number_nodes(rc_gpickle *g)
{
    const size_t nt = g->tabs.size();
    int32_t ns = 0;
    bool dense = true;
    for (auto &T : g->tabs) {
        dense = dense && T.ss >= 0 && T.qs >= 0;
        ns = std::max(ns, std::max(T.ss, T.qs) + 1);
    }
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
    std::vector<uint64_t> base((size_t)ns + 1, 0);
    for (int32_t k = 0; k < ns; k++) {
        dense = dense && gmax[k] < rc_gpickle::DENSE;
        base[k + 1] = base[k] + (uint64_t)(gmax[k] + 1);
    }
    dense = dense && base[ns] <= 4 * g->rows + (1u << 24);
    if (!dense) {
        for (auto &T : g->tabs) {
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
            T.su = Raw<uint32_t>(T.n);
            T.qu = Raw<uint32_t>(T.n);
            for (uint64_t i = 0; i < T.n; i++) T.su[i] = node_id(T.ss, T.sg[i]);
            for (uint64_t i = 0; i < T.n; i++) T.qu[i] = node_id(T.qs, T.qg[i]);
        }
        return;
    }
    const uint64_t nslot = base[ns];
    Raw<std::atomic<uint64_t>> first(nslot);
    parallel_for((nslot + 65535) / 65536, [&](size_t c) {
        for (uint64_t k = c * 65536; k < std::min<uint64_t>(nslot, (c + 1) * 65536); k++)
            first[k].store(~0ull, std::memory_order_relaxed);
    });
    // occurrence rank (table, side, row)
    parallel_for(nt, [&](size_t t) {
        const rc_gpickle::Tab &T = g->tabs[t];
        auto seen = [&](uint64_t slot, uint64_t r) {
            uint64_t cur = first[slot].load(std::memory_order_relaxed);
            while (r < cur && !first[slot].compare_exchange_weak(cur, r, std::memory_order_relaxed)) {
            }
        };
        for (uint64_t i = 0; i < T.n; i++) seen(base[T.ss] + (uint64_t)T.sg[i], ((uint64_t)t << 33) | i);
        for (uint64_t i = 0; i < T.n; i++) seen(base[T.qs] + (uint64_t)T.qg[i], ((uint64_t)t << 33) | (1ull << 32) | i);
    });
    // the occurring slots, ordered by first occurrence
    const size_t NC = (nslot + 65535) / 65536;
    std::vector<uint64_t> ccount(NC + 1, 0);
    parallel_for(NC, [&](size_t c) {
        uint64_t k0 = 0;
        for (uint64_t k = c * 65536; k < std::min<uint64_t>(nslot, (c + 1) * 65536); k++)
            k0 += first[k].load(std::memory_order_relaxed) != ~0ull;
        ccount[c + 1] = k0;
    });
    for (size_t c = 0; c < NC; c++) ccount[c + 1] += ccount[c];
    const uint64_t nn = ccount[NC];
    std::vector<std::pair<uint64_t, uint32_t>> occ(nn);   // (first rank, slot)
    parallel_for(NC, [&](size_t c) {
        uint64_t w = ccount[c];
        for (uint64_t k = c * 65536; k < std::min<uint64_t>(nslot, (c + 1) * 65536); k++) {
            const uint64_t f = first[k].load(std::memory_order_relaxed);
            if (f != ~0ull) occ[w++] = {f, (uint32_t)k};
        }
    });
    first = Raw<std::atomic<uint64_t>>();
    std::sort(occ.begin(), occ.end());
    Raw<uint32_t> id(nslot);
    g->node.resize(nn);
    parallel_for((nn + 65535) / 65536, [&](size_t c) {
        for (uint64_t k = c * 65536; k < std::min<uint64_t>(nn, (c + 1) * 65536); k++) {
            const uint32_t slot = occ[k].second;
            id[slot] = (uint32_t)k;
            const int32_t smp = (int32_t)(std::upper_bound(base.begin(), base.end(), (uint64_t)slot) - base.begin()) - 1;
            g->node[k] = NodeKey{(int64_t)(slot - base[smp]), smp};
        }
    });
    parallel_for(nt, [&](size_t t) {
        rc_gpickle::Tab &T = g->tabs[t];
        T.su = Raw<uint32_t>(T.n);
        T.qu = Raw<uint32_t>(T.n);
        for (uint64_t i = 0; i < T.n; i++) T.su[i] = id[base[T.ss] + (uint64_t)T.sg[i]];
        for (uint64_t i = 0; i < T.n; i++) T.qu[i] = id[base[T.qs] + (uint64_t)T.qg[i]];
        T.sg = Raw<int64_t>();
        T.qg = Raw<int64_t>();
    });
}

int rc_graph_pickle_write(rc_gpickle *g, const char *path, int32_t n_names, const char *const *names)
{
    if (!g || !path || (n_names && !names)) return rcg_fail(RC_E_ARG, "null argument");
    const bool tmg = getenv("RC_OUT_TIMING") && atoi(getenv("RC_OUT_TIMING"));
    auto clk = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!tmg) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "graph.pkl %s %.3f s\n", what, std::chrono::duration<double>(t - clk).count());
        clk = t;
    };
    number_nodes(g);
    lap("nodes");
    if (g->node.size() >= 0x7FFFFFFFull) return rcg_fail(RC_E_LIMIT, "graph too large for the pickle writer");
    const size_t nn = g->node.size(), nt = g->tabs.size();
    for (const NodeKey &k : g->node)
        if (k.sample < 0 || k.sample >= n_names) return rcg_fail(RC_E_ARG, "sample index out of range");
    // 1. the edges: first occurrence of each (s-node, q-node) pair, per
    // sample-pair group of tables (in call order) on its own thread
    Raw<uint8_t> keep(g->rows);
    {
        std::map<std::pair<int32_t, int32_t>, std::vector<uint32_t>> groups;
        for (size_t t = 0; t < nt; t++) groups[{g->tabs[t].lo, g->tabs[t].hi}].push_back((uint32_t)t);
        std::vector<const std::vector<uint32_t> *> gl;
        for (auto &kv : groups) gl.push_back(&kv.second);
        parallel_for(gl.size(), [&](size_t k) {
            uint64_t rows = 0;
            for (uint32_t t : *gl[k]) rows += g->tabs[t].n;
            EdgeMap em;
            while (em.key.size() < 2 * rows + 2) em.grow();
            for (uint32_t t : *gl[k]) {
                const rc_gpickle::Tab &T = g->tabs[t];
                for (uint64_t i = 0; i < T.n; i++) {
                    const uint32_t a = T.su[i], b = T.qu[i];
                    keep[T.off + i] = em.add(a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a)) ? 1 : 0;
                }
            }
        });
    }
    // edges in insertion order: tables in call order, rows in order
    std::vector<uint64_t> tcount(nt + 1, 0);
    parallel_for(nt, [&](size_t t) {
        uint64_t c = 0;
        for (uint64_t i = g->tabs[t].off; i < g->tabs[t].off + g->tabs[t].n; i++) c += keep[i];
        tcount[t + 1] = c;
    });
    for (size_t t = 0; t < nt; t++) tcount[t + 1] += tcount[t];
    const size_t ne = tcount[nt];
    struct UV {
        uint32_t first, second;
    };
    Raw<UV> edge(ne);
    parallel_for(nt, [&](size_t t) {
        const rc_gpickle::Tab &T = g->tabs[t];
        uint64_t w = tcount[t];
        for (uint64_t i = 0; i < T.n; i++)
            if (keep[T.off + i]) edge[w++] = {T.su[i], T.qu[i]};
    });
    keep = Raw<uint8_t>();
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
                h[edge[i].first / span]++;
                if (edge[i].second != edge[i].first) h[edge[i].second / span]++;
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
        lap("csr count");
        Raw<Ent> ent(bstart[NB]);
        lap("csr alloc");
        parallel_for(nec, [&](size_t c) {
            uint64_t *h = &cnt[c * NB];
            for (size_t i = c * ECH; i < std::min(ne, (c + 1) * ECH); i++) {
                const uint32_t a = edge[i].first, b2 = edge[i].second;
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
        lap("csr degrees");
        nbr = Raw<uint32_t>(off[nn]);
        eid = Raw<uint32_t>(off[nn]);
        lap("csr alloc2");
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
        const int32_t s = g->node[i].sample;
        if (name_memo[s] == 0xFFFFFFFFu) {
            name_memo[s] = (uint32_t)memo++;
            name_here[i] = 1;
        }
        node_memo[i] = (uint32_t)memo;
        memo += 2;
    }
    memo += 2;   // "_adj", its dict
    std::vector<uint64_t> adj_memo(nn + 1);
    {
        // new edge dicts per node (neighbour ids above the node, or itself)
        std::vector<uint32_t> nnew(nn, 0);
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
    }
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
    // whole SETITEMS batches written on the pool, tail; then the file
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
    const size_t CH = 64 * BATCH;   // nodes per chunk
    const size_t nch = (nn + CH - 1) / CH;
    std::vector<Out> nodes_out(nch), adj_out(nch);
    std::vector<size_t> name_len(n_names);
    for (int32_t k = 0; k < n_names; k++) name_len[k] = strlen(names[k]);
    parallel_for(2 * nch, [&](size_t x) {
        const size_t c = x % nch, i0c = c * CH, i1 = std::min(nn, (c + 1) * CH);
        if (x < nch) {
            // per node at most: a name (6 + its length) or its get (5), the
            // gene (10), TUPLE2 + memo + '}' + memo (4); per batch '(' 'u'
            size_t cap = 2 * ((i1 - i0c) / BATCH + 1);
            for (size_t i = i0c; i < i1; i++) cap += 19 + (name_here[i] ? 1 + name_len[g->node[i].sample] : 0);
            nodes_out[c] = Out(cap);
            Out &o = nodes_out[c];
            for (size_t i0 = c * CH; i0 < i1; i0 += BATCH) {
                o.op('(');
                for (size_t i = i0; i < i1 && i < i0 + BATCH; i++) {
                    const NodeKey &k = g->node[i];
                    if (name_here[i]) {
                        const uint32_t len = (uint32_t)strlen(names[k.sample]);
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
        } else {
            // per node: get + '}' + memo (7), per neighbour get + dict or get
            // (10), per batch of either '(' 'u'
            const uint64_t ents = off[i1] - off[i0c];
            adj_out[c] = Out(7 * (i1 - i0c) + 10 * ents + 2 * (ents / BATCH + 2 * (i1 - i0c) + 2));
            Out &o = adj_out[c];
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
        }
    });
    lap("stream");
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
    // the pieces at their offsets, written by the pool (pwrite: the page
    // cache copy of ~0.5 GB at C3, ~15 GB at C5, on many threads)
    std::vector<const Out *> pieces = {&head};
    for (auto &o : nodes_out) pieces.push_back(&o);
    pieces.push_back(&mid);
    for (auto &o : adj_out) pieces.push_back(&o);
    pieces.push_back(&tail);
    std::vector<uint64_t> at(pieces.size() + 1, 0);
    for (size_t k = 0; k < pieces.size(); k++) at[k + 1] = at[k] + pieces[k]->size();
    const std::string tmp = std::string(path) + ".tmp";
    const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return rcg_fail(RC_E_IO, "cannot open " + tmp);
    std::atomic<bool> werr{ftruncate(fd, (off_t)at.back()) != 0};
    parallel_for(pieces.size(), [&](size_t k) {
        const char *p = pieces[k]->buf.p.get();
        uint64_t done = 0, n = pieces[k]->size();
        while (done < n && !werr) {
            const ssize_t r = pwrite(fd, p + done, std::min<uint64_t>(n - done, 1u << 30), (off_t)(at[k] + done));
            if (r <= 0) werr = true;
            else done += (uint64_t)r;
        }
    });
    if (close(fd) != 0 || werr) {
        remove(tmp.c_str());
        return rcg_fail(RC_E_IO, "write failed: " + tmp);
    }
    if (rename(tmp.c_str(), path) != 0) return rcg_fail(RC_E_IO, std::string("cannot rename to ") + path);
    lap("file");
    return RC_OK;
}

}  // extern "C"
