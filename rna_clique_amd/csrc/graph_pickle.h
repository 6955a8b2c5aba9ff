// The graph.pkl writer's slot-form input (graph_pickle.cpp), shared with the
// engine, which hands over its device-sorted edge records in this form.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

// an array of trivially constructible T left uninitialised: its pages are
// first touched by the threads that fill it, not zeroed up front on one
// thread (hundreds of MB at C3, tens of GB at C5). Large arrays are their own
// anonymous mapping with transparent huge pages requested (2 MB pages: 512x
// fewer first-touch faults; the writer touches ~50 GB at C5)
void *raw_alloc(size_t bytes);
void raw_free(void *p, size_t bytes);

template <class T>
struct Raw {
    T *p = nullptr;
    size_t n = 0;
    Raw() = default;
    explicit Raw(size_t k) : p(k ? static_cast<T *>(raw_alloc(k * sizeof(T))) : nullptr), n(k) {}
    Raw(const Raw &) = delete;
    Raw &operator=(const Raw &) = delete;
    Raw(Raw &&o) noexcept : p(o.p), n(o.n)
    {
        o.p = nullptr;
        o.n = 0;
    }
    Raw &operator=(Raw &&o) noexcept
    {
        if (this != &o) {
            reset();
            p = o.p;
            n = o.n;
            o.p = nullptr;
            o.n = 0;
        }
        return *this;
    }
    ~Raw() { reset(); }
    void reset()
    {
        if (p) raw_free(p, n * sizeof(T));
        p = nullptr;
        n = 0;
    }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
    T *data() { return p; }
    const T *data() const { return p; }
};

struct GraphNodeKey {
    int64_t gene;
    int32_t sample;
};

// Every (sample, gene) node is a slot; the slots of sample s are
// [base[s], base[s + 1]) (gene = slot_gene[slot], or slot - base[s] when
// slot_gene is null), and each table's rows are slot pairs U[off + i]
// (s-node), V[off + i] (q-node), tables in build_graph's order. With `ids`
// set, U and V hold node ids already and `node` the nodes in insertion order.
// `unique`: no (s-node, q-node) pair repeats (the engine's edge records are
// one per edge), so the writer skips its edge deduplication.
struct GraphSlots {
    int32_t ns = 0;
    std::vector<uint64_t> base;
    const int32_t *slot_gene = nullptr;
    struct Tab {
        int32_t ss, qs;
        uint64_t off, n;
    };
    std::vector<Tab> tabs;
    uint64_t rows = 0;
    Raw<uint32_t> U, V;
    bool unique = false;
    bool ids = false;
    std::vector<GraphNodeKey> node;
};

// the whole write (RC_OK or an error code, message set); consumes G's arrays
int graph_pickle_write_slots(GraphSlots &G, const char *path, int32_t n_names, const char *const *names);
