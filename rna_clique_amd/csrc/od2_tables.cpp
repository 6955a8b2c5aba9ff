// od2 gene matches tables written natively: `{s1}--{s2}.h5` in pandas' table
// format under key "gene_matches", the file write_table (gene_matches_tables.py:
// 42-56) gives a HomologFinder table with the ssample/qsample columns of
// find_homologs_and_save (find_all_pairs.py:57-88; schema docs/formats.md:
// 231-252).
//
// The same bytes as rna_clique_amd.h5.write_frame_table(rows_to_table(rows))
// (tests/test_od2_native.py compares them; tests/test_h5_pytables.py reads the
// Python writer's files back with real PyTables + pandas): the column values
// (pident and evalue as BLAST prints them, read back), shrink_df's integer
// downcast per column, pandas' consolidated blocks (categoricals first, then
// one block per dtype in dtype-name order, columns in frame order), PyTables'
// attribute set with its protocol-0 pickles, and h5.py's classic HDF5 layout
// (superblock v0, v1 object headers, symbol-table groups, contiguous data).
// Writing natively takes the pandas frame, the per-column Python work and the
// GIL out of the tables leg of the wall clock; a pool of threads writes the
// files of many pairs at once (rc_write_tables, engine.hip).
#include "../../include/rcgpu.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

int rcg_fail(int code, const std::string &msg);

namespace od2 {

// ------------------------------------------------------------------ bytes
static void put_u8(std::string &s, unsigned v) { s.push_back((char)(uint8_t)v); }
static void put_u16(std::string &s, unsigned v)
{
    put_u8(s, v & 0xFF);
    put_u8(s, (v >> 8) & 0xFF);
}
static void put_u32(std::string &s, uint32_t v)
{
    for (int i = 0; i < 4; i++) put_u8(s, (v >> (8 * i)) & 0xFF);
}
static void put_u64(std::string &s, uint64_t v)
{
    for (int i = 0; i < 8; i++) put_u8(s, (unsigned)((v >> (8 * i)) & 0xFF));
}
static void pad8(std::string &s) { s.append((8 - s.size() % 8) % 8, '\0'); }
static std::string padded(std::string s)
{
    pad8(s);
    return s;
}

const uint64_t UNDEF = ~0ull;
const int LEAF_K = 4, INTERNAL_K = 16;

// ------------------------------------------------------------- datatypes
static std::string dt_head(unsigned cls_ver, unsigned b0, unsigned b1, unsigned b2, uint32_t size)
{
    std::string s;
    put_u8(s, cls_ver);
    put_u8(s, b0);
    put_u8(s, b1);
    put_u8(s, b2);
    put_u32(s, size);
    return s;
}
static std::string dt_int(int size, bool is_signed)
{
    std::string s = dt_head(0x10, is_signed ? 0x08 : 0, 0, 0, (uint32_t)size);
    put_u16(s, 0);
    put_u16(s, 8u * size);
    return s;
}
static std::string dt_f64()
{
    std::string s = dt_head(0x11, 0x20, 63, 0, 8);
    put_u16(s, 0);
    put_u16(s, 64);
    put_u8(s, 52);
    put_u8(s, 11);
    put_u8(s, 0);
    put_u8(s, 52);
    put_u32(s, 1023);
    return s;
}
static std::string dt_string(uint32_t size, bool utf8) { return dt_head(0x13, (utf8 ? 1u : 0u) << 4, 0, 0, size); }
static std::string dt_bitfield(int size)
{
    std::string s = dt_head(0x14, 0, 0, 0, (uint32_t)size);
    put_u16(s, 0);
    put_u16(s, 8u * size);
    return s;
}
static std::string dt_array1(uint32_t k, const std::string &base, uint32_t base_size)
{
    std::string s = dt_head(0x2A, 0, 0, 0, k * base_size);
    put_u8(s, 1);
    s.append(3, '\0');
    put_u32(s, k);
    put_u32(s, 0);
    return s + base;
}
struct Member {
    std::string name;
    uint32_t off;
    std::string dt;
};
static std::string dt_compound(const std::vector<Member> &m, uint32_t size)
{
    const size_t n = m.size();
    std::string s = dt_head(0x26, n & 0xFF, (n >> 8) & 0xFF, 0, size);
    for (const Member &x : m) {
        s += padded(x.name + std::string(1, '\0'));
        put_u32(s, x.off);
        s += x.dt;
    }
    return s;
}
static std::string dataspace(const std::vector<uint64_t> &shape)
{
    std::string s;
    put_u8(s, 1);
    put_u8(s, (unsigned)shape.size());
    put_u8(s, 0);
    put_u8(s, 0);
    s.append(4, '\0');
    for (uint64_t d : shape) put_u64(s, d);
    return s;
}

// ------------------------------------------------------------- messages
static std::string msg(unsigned type, std::string body, unsigned flags = 0)
{
    pad8(body);
    std::string s;
    put_u16(s, type);
    put_u16(s, (unsigned)body.size());
    put_u8(s, flags);
    s.append(3, '\0');
    return s + body;
}

// attribute values as h5._value makes them
struct Attr {
    std::string name;
    enum Kind { STR, BYTES, I64 } kind;
    std::string s;
    int64_t i = 0;
};
static Attr astr(const std::string &n, const std::string &v) { return Attr{n, Attr::STR, v, 0}; }
static Attr abytes(const std::string &n, const std::string &v) { return Attr{n, Attr::BYTES, v, 0}; }
static Attr ai64(const std::string &n, int64_t v) { return Attr{n, Attr::I64, "", v}; }

static std::string attr_msg(const Attr &a)
{
    std::string dt, raw;
    if (a.kind == Attr::I64) {
        dt = dt_int(8, true);
        put_u64(raw, (uint64_t)a.i);
    } else {
        raw = a.s.empty() ? std::string(1, '\0') : a.s;
        dt = dt_string((uint32_t)raw.size(), a.kind == Attr::STR);
    }
    const std::string ds = dataspace({});
    const std::string nm = a.name + std::string(1, '\0');
    std::string body;
    put_u8(body, 1);
    put_u8(body, 0);
    put_u16(body, (unsigned)nm.size());
    put_u16(body, (unsigned)dt.size());
    put_u16(body, (unsigned)ds.size());
    body += padded(nm) + padded(dt) + padded(ds) + raw;
    return msg(0x000C, body);
}
static std::string object_header(const std::vector<std::string> &msgs)
{
    std::string data;
    for (const std::string &m : msgs) data += m;
    std::string s;
    put_u8(s, 1);
    put_u8(s, 0);
    put_u16(s, (unsigned)msgs.size());
    put_u32(s, 1);
    put_u32(s, (uint32_t)data.size());
    s.append(4, '\0');
    return s + data;
}

// ------------------------------------------------------------- object tree
struct File {
    std::string buf = std::string(96, '\0');   // superblock placeholder
    uint64_t alloc(const std::string &d)
    {
        const uint64_t a = buf.size();
        buf += d;
        pad8(buf);
        return a;
    }
};

struct Node {
    bool group = true;
    std::vector<Attr> attrs;
    std::map<std::string, Node> children;   // byte order of the names, as h5.Group sorts them
    // datasets: type, shape and the raw bytes (or a writer appending them)
    std::string dt;
    std::vector<uint64_t> shape;
    std::string raw;
    uint64_t raw_size = 0;
    void (*fill)(std::string &, const void *) = nullptr;
    const void *fill_arg = nullptr;
};

static uint64_t write_node(Node &nd, File &f);

static uint64_t write_dataset(Node &d, File &f)
{
    uint64_t addr = UNDEF, size = 0;
    if (d.fill) {
        addr = f.buf.size();
        d.fill(f.buf, d.fill_arg);
        size = f.buf.size() - addr;
        if (!size) addr = UNDEF;
        pad8(f.buf);
    } else if (!d.raw.empty()) {
        addr = f.alloc(d.raw);
        size = d.raw.size();
    }
    std::string layout;
    put_u8(layout, 3);
    put_u8(layout, 1);
    put_u64(layout, addr);
    put_u64(layout, size);
    std::string fill;
    put_u8(fill, 2);
    put_u8(fill, 2);
    put_u8(fill, 2);
    put_u8(fill, 0);
    std::vector<std::string> msgs = {msg(0x0001, dataspace(d.shape)), msg(0x0003, d.dt, 1), msg(0x0005, fill, 1),
                                     msg(0x0008, layout)};
    for (const Attr &a : d.attrs) msgs.push_back(attr_msg(a));
    return f.alloc(object_header(msgs));
}

struct GroupAddr {
    uint64_t ohdr, btree, heap;
};

static GroupAddr write_group(Node &g, File &f)
{
    std::vector<std::string> names;
    for (auto &kv : g.children) names.push_back(kv.first);
    std::map<std::string, uint64_t> child_addr;
    for (const std::string &n : names) child_addr[n] = write_node(g.children[n], f);
    std::string heap(8, '\0');
    std::map<std::string, uint64_t> name_off;
    for (const std::string &n : names) {
        name_off[n] = heap.size();
        heap += padded(n + std::string(1, '\0'));
    }
    const uint64_t heap_data = f.alloc(heap);
    std::string hh = "HEAP";
    put_u8(hh, 0);
    hh.append(3, '\0');
    put_u64(hh, heap.size());
    put_u64(hh, 1);   // no free block
    put_u64(hh, heap_data);
    const uint64_t heap_addr = f.alloc(hh);
    std::string sn = "SNOD";
    put_u8(sn, 1);
    put_u8(sn, 0);
    put_u16(sn, (unsigned)names.size());
    for (const std::string &n : names) {
        put_u64(sn, name_off[n]);
        put_u64(sn, child_addr[n]);
        put_u32(sn, 0);
        put_u32(sn, 0);
        sn.append(16, '\0');
    }
    sn.append((size_t)40 * (2 * LEAF_K - names.size()), '\0');
    const uint64_t snod = f.alloc(sn);
    const int nkeys = 2 * INTERNAL_K + 1, nchild = 2 * INTERNAL_K;
    std::string bt = "TREE";
    put_u8(bt, 0);
    put_u8(bt, 0);
    put_u16(bt, names.empty() ? 0 : 1);
    put_u64(bt, UNDEF);
    put_u64(bt, UNDEF);
    if (!names.empty()) {
        put_u64(bt, 0);
        put_u64(bt, snod);
        put_u64(bt, name_off[names.back()]);
        bt.append((size_t)8 * (nkeys + nchild) - 24, '\0');
    } else {
        bt.append((size_t)8 * (nkeys + nchild), '\0');
    }
    const uint64_t btree = f.alloc(bt);
    std::string stab;
    put_u64(stab, btree);
    put_u64(stab, heap_addr);
    std::vector<std::string> msgs = {msg(0x0011, stab)};
    for (const Attr &a : g.attrs) msgs.push_back(attr_msg(a));
    return GroupAddr{f.alloc(object_header(msgs)), btree, heap_addr};
}

static uint64_t write_node(Node &nd, File &f) { return nd.group ? write_group(nd, f).ohdr : write_dataset(nd, f); }

static std::string finish_file(Node &root)
{
    File f;
    const GroupAddr r = write_group(root, f);
    const uint64_t eof = f.buf.size();
    std::string sb = "\x89HDF\r\n\x1a\n";
    const unsigned v[8] = {0, 0, 0, 0, 0, 8, 8, 0};
    for (unsigned x : v) put_u8(sb, x);
    put_u16(sb, LEAF_K);
    put_u16(sb, INTERNAL_K);
    put_u32(sb, 0);
    put_u64(sb, 0);
    put_u64(sb, UNDEF);
    put_u64(sb, eof);
    put_u64(sb, UNDEF);
    put_u64(sb, 0);
    put_u64(sb, r.ohdr);
    put_u32(sb, 1);
    put_u32(sb, 0);
    put_u64(sb, r.btree);
    put_u64(sb, r.heap);
    std::memcpy(&f.buf[0], sb.data(), 96);
    return std::move(f.buf);
}

// ------------------------------------------------------------- pickle protocol 0
// (PyTables stores Python-object attributes as protocol-0 pickles; these are
// the few shapes pandas' table attributes take: None, bool, int, ASCII str,
// list, tuple, dict -- memo numbering as pickle.dumps(obj, 0) assigns it)
struct Pk {
    std::string out;
    int memo = 0;
    // strings met again are the same (interned) Python object: pickle refers
    // back to the first with GET (e.g. the "ordered" key of every categorical)
    std::map<std::string, int> seen;
    void put() { out += "p" + std::to_string(memo++) + "\n"; }
    void none() { out += "N"; }
    void boolean(bool v) { out += v ? "I01\n" : "I00\n"; }
    void integer(long v) { out += "I" + std::to_string(v) + "\n"; }
    void str(const std::string &s)
    {
        auto it = seen.find(s);
        if (it != seen.end()) {
            out += "g" + std::to_string(it->second) + "\n";
            return;
        }
        seen[s] = memo;
        out += "V";
        for (unsigned char c : s) {
            if (c == '\\' || c == '\n' || c == '\r' || c == 0x1a || c >= 0x80) {   // raw-unicode-escape (ASCII here)
                char b[8];
                std::snprintf(b, sizeof b, "\\u%04x", c);
                out += b;
            } else {
                out += (char)c;
            }
        }
        out += "\n";
        put();
    }
    void list_begin()
    {
        out += "(l";
        out += "p" + std::to_string(memo++) + "\n";
    }
    void append() { out += "a"; }
    void dict_begin()
    {
        out += "(d";
        out += "p" + std::to_string(memo++) + "\n";
    }
    void setitem() { out += "s"; }
    void tuple_begin() { out += "("; }
    void tuple_end()
    {
        out += "t";
        put();
    }
    std::string done() { return out + "."; }
};

static std::string pk_none() { return "N."; }
static std::string pk_str_list(const std::vector<std::string> &v)
{
    Pk p;
    p.list_begin();
    for (const std::string &s : v) {
        p.str(s);
        p.append();
    }
    return p.done();
}
static std::string pk_index_cols()   // [(0, "index")]
{
    Pk p;
    p.list_begin();
    p.tuple_begin();
    p.integer(0);
    p.str("index");
    p.tuple_end();
    p.append();
    return p.done();
}
static std::string pk_non_index_axes(const std::vector<std::string> &cols)   // [(1, cols)]
{
    Pk p;
    p.list_begin();
    p.tuple_begin();
    p.integer(1);
    p.list_begin();
    for (const std::string &c : cols) {
        p.str(c);
        p.append();
    }
    p.tuple_end();
    p.append();
    return p.done();
}
// {1: {"names": [None], "type": "Index"}, "index": {}, block: {} or {"ordered": False}, ...}
static std::string pk_info(const std::vector<std::pair<std::string, int>> &blocks)   // (name, categorical)
{
    Pk p;
    p.dict_begin();
    p.integer(1);
    p.dict_begin();
    p.str("names");
    p.list_begin();
    p.none();
    p.append();
    p.setitem();
    p.str("type");
    p.str("Index");
    p.setitem();
    p.setitem();
    p.str("index");
    p.dict_begin();
    p.setitem();
    for (auto &b : blocks) {
        p.str(b.first);
        p.dict_begin();
        if (b.second) {
            p.str("ordered");
            p.boolean(false);
            p.setitem();
        }
        p.setitem();
    }
    return p.done();
}

static const std::vector<Attr> PT_GROUP = {astr("CLASS", "GROUP"), astr("TITLE", ""), astr("VERSION", "1.0")};

static std::vector<Attr> frame_attrs(const std::string &pandas_type, const std::string &table_type,
                                     const std::vector<std::string> &cols, const std::vector<std::string> &values_cols,
                                     const std::vector<std::string> &data_columns, const std::string &info)
{
    std::vector<Attr> a = PT_GROUP;
    a.push_back(abytes("data_columns", pk_str_list(data_columns)));
    a.push_back(astr("encoding", "UTF-8"));
    a.push_back(astr("errors", "strict"));
    a.push_back(abytes("index_cols", pk_index_cols()));
    a.push_back(abytes("info", info));
    a.push_back(ai64("levels", 1));
    a.push_back(astr("nan_rep", "nan"));
    a.push_back(abytes("non_index_axes", pk_non_index_axes(cols)));
    a.push_back(astr("pandas_type", pandas_type));
    a.push_back(astr("pandas_version", "0.15.2"));
    a.push_back(astr("table_type", table_type));
    a.push_back(abytes("values_cols", pk_str_list(values_cols)));
    return a;
}

static std::vector<Attr> table_attrs(uint64_t nrows)
{
    return {astr("CLASS", "TABLE"), astr("TITLE", ""), astr("VERSION", "2.7"), ai64("NROWS", (int64_t)nrows)};
}

// a Series of one string in table format: a categorical column's categories
// (h5._series_table)
struct Series1 {
    std::string v;   // the category, UTF-8
};
static void fill_series(std::string &buf, const void *arg)
{
    const Series1 *s = static_cast<const Series1 *>(arg);
    put_u64(buf, 0);   // index 0
    buf += s->v;       // S{len} value
}
static Node series_table(Series1 &s)
{
    if (s.v.empty()) s.v.assign(1, '\0');   // S1 holding b"" (h5._strings: at least 1 byte)
    const uint32_t w = (uint32_t)s.v.size();
    Node t;
    t.group = false;
    t.dt = dt_compound({{"index", 0, dt_int(8, true)}, {"values", 8, dt_string(w, false)}}, 8 + w);
    t.shape = {1};
    t.fill = fill_series;
    t.fill_arg = &s;
    t.attrs = table_attrs(1);
    t.attrs.push_back(astr("index_kind", "integer"));
    t.attrs.push_back(astr("values_dtype", "bytes" + std::to_string(8 * w)));
    t.attrs.push_back(abytes("values_kind", pk_str_list({"values"})));
    t.attrs.push_back(abytes("values_meta", pk_none()));
    Node g;
    g.attrs = frame_attrs("series_table", "appendable_series", {"values"}, {"values"}, {"values"},
                          pk_info({{"values", 0}}));
    g.children["table"] = std::move(t);
    return g;
}

// ------------------------------------------------------------- the gene matches frame
enum Col { PIDENT, LENGTH, MISMATCH, GAPOPEN, QSTART, QEND, SSTART, SEND, EVALUE, BITSCORE, GAPS, NIDENT, SSTRAND,
           QGENE, QISO, SGENE, SISO, REVERSE, SSAMPLE, QSAMPLE, NCOL };
static const char *const COL_NAMES[NCOL] = {"pident", "length", "mismatch", "gapopen", "qstart", "qend", "sstart",
                                            "send", "evalue", "bitscore", "gaps", "nident", "sstrand", "qgene",
                                            "qiso", "sgene", "siso", "reverse", "ssample", "qsample"};
static const Col INT_COLS[] = {LENGTH, MISMATCH, GAPOPEN, QSTART, QEND, SSTART, SEND, GAPS, NIDENT,
                               QGENE, QISO, SGENE, SISO};

static int64_t int_value(const rc_row &r, Col c)
{
    switch (c) {
    case LENGTH: return r.hsp.length;
    case MISMATCH: return r.hsp.mismatch;
    case GAPOPEN: return r.hsp.gapopen;
    case QSTART: return r.hsp.qstart;
    case QEND: return r.hsp.qend;
    case SSTART: return r.hsp.sstart;
    case SEND: return r.hsp.send;
    case GAPS: return r.hsp.gaps;
    case NIDENT: return r.hsp.nident;
    case QGENE: return r.qgene;
    case QISO: return r.qiso;
    case SGENE: return r.sgene;
    case SISO: return r.siso;
    default: return 0;
    }
}

// a dtype of the frame's blocks
struct DType {
    char kind;   // 'u' 'i' 'f' 'b' 'S'
    int size;
    std::string name() const
    {
        if (kind == 'f') return "float64";
        if (kind == 'b') return "bool";
        if (kind == 'S') return "object";   // the block's pandas dtype (its values are written as S)
        return std::string(kind == 'u' ? "uint" : "int") + std::to_string(8 * size);
    }
    std::string h5() const
    {
        if (kind == 'f') return dt_f64();
        if (kind == 'b') return dt_bitfield(1);
        if (kind == 'S') return dt_string((uint32_t)size, false);
        return dt_int(size, kind == 'i');
    }
};

// shrink_df's downcast (tables.downcast_int): the smallest unsigned type when
// no value is negative, else the smallest signed one; an empty column uint8
static DType downcast(int64_t mn, int64_t mx, bool empty)
{
    if (empty) return DType{'u', 1};
    if (mn >= 0) {
        for (int s : {1, 2, 4, 8})
            if (s == 8 || (uint64_t)mx <= (1ull << (8 * s)) - 1) return DType{'u', s};
    }
    for (int s : {1, 2, 4, 8})
        if (s == 8 || (mn >= -(1ll << (8 * s - 1)) && mx <= (1ll << (8 * s - 1)) - 1)) return DType{'i', s};
    return DType{'i', 8};
}

struct Block {
    DType dt;
    std::vector<Col> cols;
    bool categorical = false;
};

struct Table {
    const rc_row *rows;
    uint64_t n;
    std::vector<double> pident, evalue, bits;
    // the frame's columns, gathered once from the rows (fill_records writes
    // them column by column into cache-sized runs of records)
    std::vector<int32_t> ic[NCOL], label;
    std::vector<uint8_t> rev, minus;
    DType coldt[NCOL];
    std::vector<Block> blocks;
    std::vector<uint32_t> boff;   // record offset of each block
    uint32_t rec = 0;
    Series1 cats[2];
};

// BLAST's tabular printing read back (tables.blast_pident / blast_evalue)
static double printed(const char *fmt, double v)
{
    char b[64];
    std::snprintf(b, sizeof b, fmt, v);
    return std::strtod(b, nullptr);
}

// one column of a run of records: v[i] into rec i at byte offset `off`, as
// the low `size` bytes of its little-endian value
template <class T, class S>
static void put_col(char *out, size_t rec, size_t off, const S *v, uint64_t i0, uint64_t i1)
{
    for (uint64_t i = i0; i < i1; i++) {
        const T x = (T)v[i];
        std::memcpy(out + i * rec + off, &x, sizeof(T));
    }
}

static void fill_records(std::string &buf, const void *arg)
{
    const Table &t = *static_cast<const Table *>(arg);
    const size_t base = buf.size(), rec = t.rec;
    buf.resize(base + rec * t.n);
    char *out = &buf[base];
    // runs of 256 records (about 20 KB: they stay in L1 while every column
    // of the run is written)
    for (uint64_t i0 = 0; i0 < t.n; i0 += 256) {
        const uint64_t i1 = std::min<uint64_t>(t.n, i0 + 256);
        put_col<int64_t>(out, rec, 0, t.label.data(), i0, i1);
        for (size_t k = 0; k < t.blocks.size(); k++) {
            const Block &b = t.blocks[k];
            size_t off = t.boff[k];
            for (Col c : b.cols) {
                const int sz = b.dt.size;
                switch (b.dt.kind) {
                case 'f': {
                    const double *v = c == PIDENT ? t.pident.data() : c == EVALUE ? t.evalue.data() : t.bits.data();
                    put_col<double>(out, rec, off, v, i0, i1);
                    break;
                }
                case 'b': put_col<uint8_t>(out, rec, off, t.rev.data(), i0, i1); break;
                case 'S':
                    for (uint64_t i = i0; i < i1; i++) {
                        char *q = out + i * rec + off;
                        const char *sv = t.minus[i] ? "minus" : "plus";
                        std::memset(q, 0, (size_t)sz);
                        std::memcpy(q, sv, std::min<size_t>(std::strlen(sv), (size_t)sz));
                    }
                    break;
                default:
                    if (b.categorical) {   // the one category's code
                        for (uint64_t i = i0; i < i1; i++) out[i * rec + off] = 0;
                    } else {
                        const int32_t *v = t.ic[c].data();
                        if (sz == 1) put_col<uint8_t>(out, rec, off, v, i0, i1);
                        else if (sz == 2) put_col<uint16_t>(out, rec, off, v, i0, i1);
                        else if (sz == 4) put_col<uint32_t>(out, rec, off, v, i0, i1);
                        else put_col<int64_t>(out, rec, off, v, i0, i1);
                    }
                }
                off += (size_t)sz;
            }
        }
    }
}

static std::string build_table_file(Table &t, const std::string &ssample, const std::string &qsample)
{
    const uint64_t n = t.n;
    // column dtypes
    t.coldt[PIDENT] = t.coldt[EVALUE] = t.coldt[BITSCORE] = DType{'f', 8};
    t.coldt[REVERSE] = DType{'b', 1};
    uint64_t nminus = 0;
    for (uint64_t i = 0; i < n; i++) nminus += t.minus[i];
    t.coldt[SSTRAND] = DType{'S', nminus ? 5 : (n ? 4 : 1)};
    for (Col c : INT_COLS) {
        const int32_t *v = t.ic[c].data();
        int32_t mn = n ? v[0] : 0, mx = mn;
        for (uint64_t i = 1; i < n; i++) {
            mn = v[i] < mn ? v[i] : mn;
            mx = v[i] > mx ? v[i] : mx;
        }
        t.coldt[c] = downcast(mn, mx, n == 0);
    }
    t.coldt[SSAMPLE] = t.coldt[QSAMPLE] = DType{'i', 1};
    // consolidated blocks: the two categoricals, then the others by dtype name
    // (pandas sorts on (can consolidate, dtype name)), columns in frame order
    t.blocks.clear();
    t.blocks.push_back(Block{DType{'i', 1}, {SSAMPLE}, true});
    t.blocks.push_back(Block{DType{'i', 1}, {QSAMPLE}, true});
    std::map<std::string, Block> byname;
    for (int c = 0; c < NCOL; c++) {
        if (c == SSAMPLE || c == QSAMPLE) continue;
        const DType d = t.coldt[c];
        Block &b = byname[d.name()];
        b.dt = d;
        if (d.kind == 'S') b.dt.size = d.size;
        b.cols.push_back((Col)c);
    }
    for (auto &kv : byname) t.blocks.push_back(kv.second);
    // the records: index int64, then each block as an array member
    std::vector<Member> mem = {{"index", 0, dt_int(8, true)}};
    uint32_t off = 8;
    t.boff.clear();
    std::vector<std::pair<std::string, int>> info_blocks;
    std::vector<std::string> names;
    Node tab;
    tab.group = false;
    tab.attrs = table_attrs(n);
    tab.attrs.push_back(astr("index_kind", "integer"));
    for (size_t k = 0; k < t.blocks.size(); k++) {
        const Block &b = t.blocks[k];
        const std::string nm = "values_block_" + std::to_string(k);
        names.push_back(nm);
        info_blocks.push_back({nm, b.categorical ? 1 : 0});
        const uint32_t kk = (uint32_t)b.cols.size();
        mem.push_back({nm, off, dt_array1(kk, b.dt.h5(), (uint32_t)b.dt.size)});
        t.boff.push_back(off);
        off += kk * (uint32_t)b.dt.size;
        std::vector<std::string> items;
        for (Col c : b.cols) items.push_back(COL_NAMES[c]);
        tab.attrs.push_back(abytes(nm + "_kind", pk_str_list(items)));
        // the values' dtype name (an object block is written as S{width})
        tab.attrs.push_back(astr(nm + "_dtype", b.dt.kind == 'S' ? "bytes" + std::to_string(8 * b.dt.size) : b.dt.name()));
        if (b.categorical) tab.attrs.push_back(astr(nm + "_meta", "category"));
        else tab.attrs.push_back(abytes(nm + "_meta", pk_none()));
    }
    t.rec = off;
    tab.dt = dt_compound(mem, off);
    tab.shape = {n};
    tab.fill = fill_records;
    tab.fill_arg = &t;
    std::vector<std::string> cols;
    for (int c = 0; c < NCOL; c++) cols.push_back(COL_NAMES[c]);
    Node frame;
    frame.attrs = frame_attrs("frame_table", "appendable_frame", cols, names, {}, pk_info(info_blocks));
    frame.children["table"] = std::move(tab);
    t.cats[0].v = ssample;
    t.cats[1].v = qsample;
    Node meta;
    meta.attrs = PT_GROUP;
    for (int k = 0; k < 2; k++) {
        Node m;
        m.attrs = PT_GROUP;
        m.children["meta"] = series_table(t.cats[k]);
        meta.children[names[k]] = std::move(m);
    }
    frame.children["meta"] = std::move(meta);
    Node root;
    root.attrs = PT_GROUP;
    root.attrs.push_back(astr("PYTABLES_FORMAT_VERSION", "2.1"));
    root.children["gene_matches"] = std::move(frame);
    return finish_file(root);
}

}  // namespace od2

// The table file of one pair's rows (rc_pair_rows order), written atomically
// (path + ".tmp", then renamed). Thread-safe: no shared state.
int od2_write_table(const rc_row *rows, uint64_t n, const std::string &ssample, const std::string &qsample,
                    const std::string &path)
{
    od2::Table t;
    t.rows = rows;
    t.n = n;
    t.pident.resize(n);
    t.evalue.resize(n);
    t.bits.resize(n);
    t.label.resize(n);
    t.rev.resize(n);
    t.minus.resize(n);
    for (od2::Col c : od2::INT_COLS) t.ic[c].resize(n);
    using namespace od2;
    int32_t *cl = t.ic[LENGTH].data(), *cm = t.ic[MISMATCH].data(), *cg = t.ic[GAPOPEN].data(),
            *cqs = t.ic[QSTART].data(), *cqe = t.ic[QEND].data(), *css = t.ic[SSTART].data(),
            *cse = t.ic[SEND].data(), *cgp = t.ic[GAPS].data(), *cni = t.ic[NIDENT].data(),
            *cqg = t.ic[QGENE].data(), *cqi = t.ic[QISO].data(), *csg = t.ic[SGENE].data(), *csi = t.ic[SISO].data();
    for (uint64_t i = 0; i < n; i++) {
        const rc_row &r = rows[i];
        cl[i] = r.hsp.length; cm[i] = r.hsp.mismatch; cg[i] = r.hsp.gapopen;
        cqs[i] = r.hsp.qstart; cqe[i] = r.hsp.qend; css[i] = r.hsp.sstart; cse[i] = r.hsp.send;
        cgp[i] = r.hsp.gaps; cni[i] = r.hsp.nident;
        cqg[i] = r.qgene; cqi[i] = r.qiso; csg[i] = r.sgene; csi[i] = r.siso;
        t.bits[i] = r.hsp.bits10 / 10.0;
        t.label[i] = r.label;
        t.rev[i] = r.reverse ? 1 : 0;
        t.minus[i] = r.hsp.strand ? 1 : 0;
    }
    // few distinct (nident, length) pairs and e-values recur over a run's
    // tables: each is printed and parsed once per thread, through a
    // direct-mapped cache kept across the thread's tables (as tables.py does
    // with np.unique per table; the values are pure functions of the key)
    struct Memo {
        uint64_t key[1 << 16];
        double val[1 << 16];
        Memo() { std::fill(key, key + (1 << 16), ~0ull); }
    };
    static thread_local std::unique_ptr<Memo> pm, em;
    if (!pm) pm.reset(new Memo());
    if (!em) em.reset(new Memo());
    auto slot = [](uint64_t k) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 48); };
    for (uint64_t i = 0; i < n; i++) {
        const rc_hsp &h = rows[i].hsp;
        const uint64_t pk = ((uint64_t)(uint32_t)h.nident << 32) | (uint32_t)h.length;
        const size_t ps = slot(pk);
        if (pm->key[ps] != pk) {
            const double L = (double)(h.length > 1 ? h.length : 1);
            pm->val[ps] = od2::printed("%.3f", 100.0 * (double)h.nident / L);
            pm->key[ps] = pk;
        }
        t.pident[i] = pm->val[ps];
        if (h.evalue < 1.0e-180) {
            t.evalue[i] = 0.0;
        } else {
            uint64_t ek;
            std::memcpy(&ek, &h.evalue, 8);
            const size_t es = slot(ek);
            if (em->key[es] != ek) {
                em->val[es] = od2::printed("%.2e", h.evalue);
                em->key[es] = ek;
            }
            t.evalue[i] = em->val[es];
        }
    }
    const std::string file = od2::build_table_file(t, ssample, qsample);
    const std::string tmp = path + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return rcg_fail(RC_E_IO, "cannot open " + tmp);
    const bool ok = std::fwrite(file.data(), 1, file.size(), f) == file.size();
    if (std::fclose(f) != 0 || !ok) {
        std::remove(tmp.c_str());
        return rcg_fail(RC_E_IO, "write failed: " + tmp);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) return rcg_fail(RC_E_IO, "cannot rename to " + path);
    return RC_OK;
}

extern "C" int rc_table_write_rows(const rc_row *rows, uint64_t n, const char *ssample, const char *qsample,
                                   const char *path)
{
    if ((n && !rows) || !ssample || !qsample || !path) return rcg_fail(RC_E_ARG, "null argument");
    return od2_write_table(rows, n, ssample, qsample, path);
}
