// TensorFlow checkpoint-V2 ("tensor bundle") reader, host-only C++ (ckpt.cpp).
//
// A V2 checkpoint <prefix> is <prefix>.index — an SSTable (LevelDB table format: prefix-
// compressed key blocks with restart points, an index block of block handles, a 48-byte footer
// with magic 0xdb4775248b80fb57) mapping each variable name to a BundleEntryProto (dtype,
// shape, shard, offset, size, masked CRC-32C), with the BundleHeaderProto under the empty key —
// and <prefix>.data-NNNNN-of-MMMMM shards holding the raw little-endian tensor bytes.  This is
// what tf.train.Saver.restore reads for methods.py:79-84.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace ast {

// largest element count a tensor entry may declare (2^40: far above any encoder variable,
// far below int64 overflow of elements x bytes)
constexpr int64_t kMaxElements = (int64_t)1 << 40;

enum CkptDtype { CK_FLOAT = 1, CK_DOUBLE = 2, CK_INT32 = 3, CK_INT64 = 9, CK_BF16 = 14, CK_HALF = 19 };

struct CkptEntry {
    std::string name;
    int dtype = 0;
    std::vector<int64_t> shape;
    int shard = 0;
    uint64_t offset = 0, size = 0;
    uint32_t crc = 0;
    bool has_crc = false;
    bool sliced = false;
    int64_t elements() const;   // -1 for a negative dim or a count above kMaxElements
};

struct Checkpoint {
    std::string prefix;
    int num_shards = 1;
    std::vector<CkptEntry> entries;   // sorted by name (table order)

    // 0 on success; otherwise a message in *err
    int open(const std::string& prefix, std::string* err);
    const CkptEntry* find(const std::string& name) const;
    // the entry's tensor as float32 (float / double / half / bfloat16 converted), checking
    // size and CRC; dst holds elements() floats
    int read_f32(const CkptEntry& e, float* dst, std::string* err) const;
};

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t init = 0);
uint32_t crc_mask(uint32_t c);

}  // namespace ast
