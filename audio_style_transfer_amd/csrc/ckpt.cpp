// TensorFlow checkpoint-V2 reader (see ckpt.h) and its C ABI (include/astyle.h: ast_ckpt_*).
// Host code only; ast_restore, which feeds ast_set_weight, lives in api.hip.
#include "ckpt.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>

namespace ast {

int set_error(int code, const std::string& msg);   // api.hip

namespace {

uint32_t g_crc_table[256];
bool g_crc_init = false;

void crc_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        g_crc_table[i] = c;
    }
    g_crc_init = true;
}

bool read_file(const std::string& path, std::string* out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    const std::streamoff n = f.tellg();
    f.seekg(0, std::ios::beg);
    out->resize((size_t)n);
    if (n > 0) f.read(&(*out)[0], n);
    return (bool)f;
}

uint32_t fixed32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// protobuf / table varints; false on truncation
bool varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
    uint64_t r = 0;
    for (int s = 0; s < 64 && p < end; s += 7) {
        const uint8_t b = *p++;
        r |= (uint64_t)(b & 0x7F) << s;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}

struct Handle {
    uint64_t offset = 0, size = 0;
};

bool decode_handle(const uint8_t*& p, const uint8_t* end, Handle* h) {
    return varint(p, end, &h->offset) && varint(p, end, &h->size);
}

// one protobuf field: number, wire type, varint value or [ptr, len) payload
struct Field {
    int num = 0, wire = 0;
    uint64_t v = 0;
    const uint8_t* p = nullptr;
    size_t n = 0;
};

bool next_field(const uint8_t*& p, const uint8_t* end, Field* f) {
    uint64_t key;
    if (!varint(p, end, &key)) return false;
    f->num = (int)(key >> 3);
    f->wire = (int)(key & 7);
    switch (f->wire) {
        case 0: return varint(p, end, &f->v);
        case 1: if (end - p < 8) return false; f->p = p; f->n = 8; p += 8; return true;
        case 5: if (end - p < 4) return false; f->p = p; f->n = 4; f->v = fixed32(p); p += 4; return true;
        case 2: {
            uint64_t n;
            if (!varint(p, end, &n) || (uint64_t)(end - p) < n) return false;
            f->p = p; f->n = (size_t)n; p += n;
            return true;
        }
        default: return false;
    }
}

// a table block (after its trailer was checked): entries with shared-prefix keys, restarts
bool parse_block(const uint8_t* b, size_t n, std::vector<std::pair<std::string, std::string>>* out,
                 std::string* err) {
    if (n < 4) { *err = "block too small"; return false; }
    const uint32_t nr = fixed32(b + n - 4);
    if ((uint64_t)nr * 4 + 4 > n) { *err = "bad restart count"; return false; }
    const uint8_t* p = b;
    const uint8_t* end = b + n - 4 - 4 * (size_t)nr;
    std::string key;
    while (p < end) {
        uint64_t shared, nonshared, vlen;
        if (!varint(p, end, &shared) || !varint(p, end, &nonshared) || !varint(p, end, &vlen) ||
            shared > key.size() || nonshared > (uint64_t)(end - p) ||
            vlen > (uint64_t)(end - p) - nonshared) {
            *err = "corrupt block entry";
            return false;
        }
        key.resize((size_t)shared);
        key.append((const char*)p, (size_t)nonshared);
        p += nonshared;
        out->emplace_back(key, std::string((const char*)p, (size_t)vlen));
        p += vlen;
    }
    return true;
}

bool read_block(const std::string& file, const Handle& h, std::string* contents, std::string* err) {
    // overflow-safe form of offset + size + 5 (trailer) <= file size: both come from the file
    const uint64_t fs = file.size();
    if (h.size > fs || fs - h.size < 5 || h.offset > fs - h.size - 5) {
        *err = "block handle past the end of the index";
        return false;
    }
    const uint8_t* b = (const uint8_t*)file.data() + h.offset;
    const uint8_t type = b[h.size];
    const uint32_t want = fixed32(b + h.size + 1);
    const uint32_t got = crc_mask(crc32c(&type, 1, crc32c(b, (size_t)h.size)));
    if (want != got) { *err = "index block CRC mismatch"; return false; }
    if (type != 0) {
        *err = "compressed table block (type " + std::to_string(type) +
               "): TF's tensor bundle writes uncompressed blocks";
        return false;
    }
    contents->assign((const char*)b, (size_t)h.size);
    return true;
}

bool parse_entry(const std::string& key, const std::string& val, CkptEntry* e, std::string* err) {
    e->name = key;
    const uint8_t* p = (const uint8_t*)val.data();
    const uint8_t* end = p + val.size();
    Field f;
    while (p < end) {
        if (!next_field(p, end, &f)) { *err = "corrupt BundleEntryProto for " + key; return false; }
        if (f.num == 1 && f.wire == 0) e->dtype = (int)f.v;
        else if (f.num == 2 && f.wire == 2) {                       // TensorShapeProto
            const uint8_t* q = f.p;
            const uint8_t* qe = f.p + f.n;
            Field g;
            while (q < qe) {
                if (!next_field(q, qe, &g)) { *err = "corrupt shape of " + key; return false; }
                if (g.num == 2 && g.wire == 2) {                    // Dim
                    const uint8_t* r = g.p;
                    const uint8_t* re = g.p + g.n;
                    Field h;
                    uint64_t size = 0;
                    while (r < re) {
                        if (!next_field(r, re, &h)) { *err = "corrupt dim of " + key; return false; }
                        if (h.num == 1 && h.wire == 0) size = h.v;
                    }
                    // a dim is an int64 >= 0; the element count must stay far from overflow
                    if (size > kMaxElements || e->shape.size() >= 32) {
                        *err = "implausible shape for " + key;
                        return false;
                    }
                    e->shape.push_back((int64_t)size);
                    if (e->elements() < 0) { *err = "implausible shape for " + key; return false; }
                } else if (g.num == 3 && g.wire == 0 && g.v) {
                    *err = "unknown-rank shape for " + key;
                    return false;
                }
            }
        } else if (f.num == 3 && f.wire == 0) e->shard = (int)f.v;
        else if (f.num == 4 && f.wire == 0) e->offset = f.v;
        else if (f.num == 5 && f.wire == 0) e->size = f.v;
        else if (f.num == 6 && f.wire == 5) { e->crc = (uint32_t)f.v; e->has_crc = true; }
        else if (f.num == 7) e->sliced = true;
    }
    return true;
}

int dtype_bytes(int dt) {
    switch (dt) {
        case CK_FLOAT: case CK_INT32: return 4;
        case CK_DOUBLE: case CK_INT64: return 8;
        case CK_BF16: case CK_HALF: return 2;
        default: return 0;
    }
}

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16;
    const int e = (h >> 10) & 0x1F;
    uint32_t m = h & 0x3FF;
    uint32_t bits;
    if (e == 0) {
        if (!m) bits = s;
        else {                                  // subnormal: normalise
            int k = -1;
            do { ++k; m <<= 1; } while (!(m & 0x400));
            bits = s | ((uint32_t)(127 - 15 - k) << 23) | ((m & 0x3FF) << 13);
        }
    } else if (e == 31) bits = s | 0x7F800000u | (m << 13);
    else bits = s | ((uint32_t)(e - 15 + 127) << 23) | (m << 13);
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

}  // namespace

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t init) {
    if (!g_crc_init) crc_init();
    uint32_t c = ~init;
    for (size_t i = 0; i < n; ++i) c = g_crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

int64_t CkptEntry::elements() const {
    int64_t n = 1;
    for (int64_t d : shape) {
        if (d < 0 || (d > 0 && n > kMaxElements / d)) return -1;   // invalid or past the cap
        n *= d;
    }
    return n;
}

int Checkpoint::open(const std::string& pre, std::string* err) {
    prefix = pre;
    entries.clear();
    std::string idx;
    if (!read_file(pre + ".index", &idx)) { *err = "cannot read " + pre + ".index"; return -1; }
    if (idx.size() < 48) { *err = pre + ".index: shorter than a table footer"; return -1; }
    const uint8_t* ft = (const uint8_t*)idx.data() + idx.size() - 48;
    const uint64_t magic = (uint64_t)fixed32(ft + 40) | ((uint64_t)fixed32(ft + 44) << 32);
    if (magic != 0xdb4775248b80fb57ull) { *err = pre + ".index: not a TF table (bad magic)"; return -1; }
    const uint8_t* p = ft;
    Handle meta, index;
    if (!decode_handle(p, ft + 40, &meta) || !decode_handle(p, ft + 40, &index)) {
        *err = pre + ".index: corrupt footer";
        return -1;
    }
    std::string blk;
    std::vector<std::pair<std::string, std::string>> ikv;
    if (!read_block(idx, index, &blk, err) ||
        !parse_block((const uint8_t*)blk.data(), blk.size(), &ikv, err)) {
        *err = pre + ".index: " + *err;
        return -1;
    }
    bool have_header = false;
    for (const auto& kv : ikv) {
        const uint8_t* q = (const uint8_t*)kv.second.data();
        Handle h;
        if (!decode_handle(q, q + kv.second.size(), &h)) { *err = pre + ".index: corrupt index entry"; return -1; }
        std::vector<std::pair<std::string, std::string>> kvs;
        if (!read_block(idx, h, &blk, err) ||
            !parse_block((const uint8_t*)blk.data(), blk.size(), &kvs, err)) {
            *err = pre + ".index: " + *err;
            return -1;
        }
        for (const auto& e : kvs) {
            if (e.first.empty()) {                                   // BundleHeaderProto
                const uint8_t* r = (const uint8_t*)e.second.data();
                const uint8_t* re = r + e.second.size();
                Field f;
                while (r < re) {
                    if (!next_field(r, re, &f)) { *err = "corrupt bundle header"; return -1; }
                    if (f.num == 1 && f.wire == 0) {
                        if (f.v < 1 || f.v > 99999) { *err = "bad shard count in bundle header"; return -1; }
                        num_shards = (int)f.v;
                    }
                    if (f.num == 2 && f.wire == 0 && f.v != 0) {
                        *err = "big-endian checkpoint";
                        return -1;
                    }
                }
                have_header = true;
                continue;
            }
            CkptEntry ce;
            if (!parse_entry(e.first, e.second, &ce, err)) return -1;
            entries.push_back(std::move(ce));
        }
    }
    if (!have_header) { *err = pre + ".index: no bundle header (not a V2 checkpoint)"; return -1; }
    std::sort(entries.begin(), entries.end(),
              [](const CkptEntry& a, const CkptEntry& b) { return a.name < b.name; });
    return 0;
}

const CkptEntry* Checkpoint::find(const std::string& name) const {
    auto it = std::lower_bound(entries.begin(), entries.end(), name,
                               [](const CkptEntry& e, const std::string& n) { return e.name < n; });
    return it != entries.end() && it->name == name ? &*it : nullptr;
}

int Checkpoint::read_f32(const CkptEntry& e, float* dst, std::string* err) const {
    if (e.sliced) { *err = e.name + ": partitioned (sliced) variables are not supported"; return -1; }
    const int eb = dtype_bytes(e.dtype);
    if (!eb || e.dtype == CK_INT32 || e.dtype == CK_INT64) {
        *err = e.name + ": dtype " + std::to_string(e.dtype) + " is not a floating-point tensor";
        return -1;
    }
    const int64_t n = e.elements();
    if (n < 0 || (uint64_t)n * eb != e.size) { *err = e.name + ": size does not match shape and dtype"; return -1; }
    if (e.shard < 0 || e.shard >= num_shards) { *err = e.name + ": shard index out of range"; return -1; }
    char fn[48];
    std::snprintf(fn, sizeof fn, ".data-%05d-of-%05d", e.shard, num_shards);
    std::ifstream f(prefix + fn, std::ios::binary);
    if (!f) { *err = "cannot read " + prefix + fn; return -1; }
    f.seekg(0, std::ios::end);
    const uint64_t fsz = (uint64_t)f.tellg();
    if (e.offset > fsz || e.size > fsz - e.offset) { *err = e.name + ": data shard shorter than its entry"; return -1; }
    std::vector<uint8_t> buf((size_t)e.size);
    f.seekg((std::streamoff)e.offset);
    if (e.size) f.read((char*)buf.data(), (std::streamsize)e.size);
    if (!f) { *err = e.name + ": data shard shorter than its entry"; return -1; }
    if (e.has_crc && crc_mask(crc32c(buf.data(), buf.size())) != e.crc) {
        *err = e.name + ": data CRC mismatch";
        return -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* q = buf.data() + i * eb;
        switch (e.dtype) {
            case CK_FLOAT: std::memcpy(dst + i, q, 4); break;
            case CK_DOUBLE: { double d; std::memcpy(&d, q, 8); dst[i] = (float)d; break; }
            case CK_HALF: dst[i] = half_to_float((uint16_t)(q[0] | (q[1] << 8))); break;
            case CK_BF16: {
                const uint32_t bits = ((uint32_t)q[0] << 16) | ((uint32_t)q[1] << 24);
                std::memcpy(dst + i, &bits, 4);
                break;
            }
        }
    }
    return 0;
}

}  // namespace ast

struct ast_ckpt {
    ast::Checkpoint ck;
};

extern "C" {

int ast_ckpt_open(const char* prefix, ast_ckpt** out) {
    if (!prefix || !out) return ast::set_error(-1, "ast_ckpt_open: null argument");
    try {   // nothing may unwind through the C ABI (bad_alloc on a hostile file included)
        std::unique_ptr<ast_ckpt> c(new ast_ckpt);
        std::string err;
        if (c->ck.open(prefix, &err)) return ast::set_error(-4, err);
        *out = c.release();
        return 0;
    } catch (const std::exception& ex) {
        return ast::set_error(-1, std::string("ast_ckpt_open: ") + ex.what());
    }
}

void ast_ckpt_close(ast_ckpt* c) { delete c; }

int ast_ckpt_num_entries(const ast_ckpt* c) { return c ? (int)c->ck.entries.size() : -1; }

int ast_ckpt_entry(const ast_ckpt* c, int i, char* name, size_t name_cap, int* dtype, int* ndim,
                   int64_t* dims, int max_dims) {
    if (!c || i < 0 || i >= (int)c->ck.entries.size())
        return ast::set_error(-1, "ast_ckpt_entry: index out of range");
    const ast::CkptEntry& e = c->ck.entries[(size_t)i];
    if (name) {
        if (name_cap < e.name.size() + 1) return ast::set_error(-1, "ast_ckpt_entry: name buffer too small");
        std::memcpy(name, e.name.c_str(), e.name.size() + 1);
    }
    if (dtype) *dtype = e.dtype;
    if (ndim) *ndim = (int)e.shape.size();
    if (dims) {
        if ((int)e.shape.size() > max_dims) return ast::set_error(-1, "ast_ckpt_entry: too many dims");
        for (size_t k = 0; k < e.shape.size(); ++k) dims[k] = e.shape[k];
    }
    return 0;
}

int ast_ckpt_read_f32(const ast_ckpt* c, const char* name, float* host, size_t n) {
    if (!c || !name || (!host && n)) return ast::set_error(-1, "ast_ckpt_read_f32: null argument");
    const ast::CkptEntry* e = c->ck.find(name);
    if (!e) return ast::set_error(-4, std::string("ast_ckpt_read_f32: no tensor named ") + name);
    if (e->elements() < 0 || (size_t)e->elements() != n)
        return ast::set_error(-1, std::string(name) + ": has " + std::to_string(e->elements()) +
                                      " elements, buffer holds " + std::to_string(n));
    try {
        std::string err;
        if (c->ck.read_f32(*e, host, &err)) return ast::set_error(-1, err);
        return 0;
    } catch (const std::exception& ex) {
        return ast::set_error(-1, std::string("ast_ckpt_read_f32: ") + ex.what());
    }
}

}  // extern "C"
