// kge_tfrecord.cpp — TF-free reader and writer of the reference's on-disk training batches
// (SURVEY §8f rank 4). Host memory only.
//
// The reference writes one tf.train.Example per batch (compress_data/main.py:117-131 with
// compress_data/utils.py:35-42) holding four flat lists:
//   "positive_sample"    Int64List  [B*3]   (np.hstack of the [B,3] batch)
//   "negative_sample"    Int64List  [B*N]
//   "subsampling_weight" FloatList  [B]     ([B,1] hstacked)
//   "mode"               Int64List  [B]
// and reads them back with tf.data.TFRecordDataset + VarLenFeature + reshape
// (tensorflow_codes/run.py:40-66, compress_data/loading_tfrecord.py:5-31).
//
// File framing (TFRecord): per record
//   uint64 length (LE) | uint32 masked_crc32c(length bytes) | data[length] | uint32 masked_crc32c(data)
// masked_crc(c) = ((c >> 15) | (c << 17)) + 0xa282ead8, CRC-32C (Castagnoli, reflected 0x82F63B78).
//
// Example proto (tensorflow/core/example/{example,feature}.proto, proto3):
//   Example   { Features features = 1; }
//   Features  { map<string, Feature> feature = 1; }      // map entry: { string key = 1; Feature value = 2; }
//   Feature   { oneof kind { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
//   FloatList { repeated float value = 1 [packed = true]; }
//   Int64List { repeated int64 value = 1 [packed = true]; }
// The parser accepts packed and unpacked repeated fields, any map order and unknown fields (skipped),
// as protobuf parsers must. The writer emits the map keys sorted (protobuf's deterministic order)
// with packed lists.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "kge_hip.h"

namespace kge_impl {
int set_error(int code, const char* msg);  // kge_abi.hip
}

namespace {

using kge_impl::set_error;

// ---- CRC-32C, slicing-by-8 ---------------------------------------------------------------------
struct Crc32cTables {
    uint32_t t[8][256];
    Crc32cTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
};
const Crc32cTables& crc_tables() {
    static const Crc32cTables tab;
    return tab;
}

#if defined(__x86_64__)
// SSE4.2's crc32 instruction computes CRC-32C itself (same polynomial, reflected): three independent
// streams over thirds of the buffer hide the instruction's 3-cycle latency, then the three CRCs are
// combined by feeding zero-extended shifts through the table-driven shift operator below.
__attribute__((target("sse4.2"))) uint32_t crc32c_hw_run(uint32_t c, const uint8_t* p, size_t n) {
    uint64_t c64 = c;
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c64 = __builtin_ia32_crc32di(c64, v);
        p += 8;
        n -= 8;
    }
    c = (uint32_t)c64;
    while (n--) c = __builtin_ia32_crc32qi(c, *p++);
    return c;
}
bool have_sse42() {
    static const bool ok = __builtin_cpu_supports("sse4.2");
    return ok;
}
#endif

uint32_t crc32c_sw_run(uint32_t c, const uint8_t* p, size_t n) {
    const auto& T = crc_tables().t;
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
            T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xFF];
    return c;
}

uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
    if (have_sse42()) return crc32c_hw_run(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu;
#endif
    return crc32c_sw_run(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu;
}

uint32_t masked_crc(const uint8_t* p, size_t n) {
    const uint32_t c = crc32c(p, n);
    return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ---- protobuf wire format ----------------------------------------------------------------------
struct Cursor {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;

    bool more() const { return ok && p < end; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int shift = 0; shift < 64; shift += 7) {
            if (p >= end) break;
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << shift;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    Cursor sub() {  // length-delimited payload
        const uint64_t n = varint();
        Cursor c{p, p, ok};
        if (!ok || n > (uint64_t)(end - p)) {
            ok = false;
            c.ok = false;
            return c;
        }
        c.end = p + n;
        p += n;
        return c;
    }
    void skip(uint32_t wire) {
        switch (wire) {
            case 0: varint(); break;
            case 1: advance(8); break;
            case 2: sub(); break;
            case 5: advance(4); break;
            default: ok = false;
        }
    }
    void advance(size_t n) {
        if (n > (size_t)(end - p)) ok = false;
        else p += n;
    }
};

// Packed varint lists (Int64List, the bulk of every record): the value count is the number of bytes
// without the continuation bit (8 bytes at a time, hardware popcount), the output is sized once, and
// values of up to 4 bytes (< 2^28: every entity id) decode branch-free from one 8-byte load: the
// first clear continuation bit gives the length, the 7-bit groups are compacted with shifts and
// masked to that length. Longer varints (negative or huge values) and the last 7 bytes take the
// careful path. A truncated or over-long last varint leaves the cursor short of / past the end, which
// is rejected.
#if defined(__x86_64__)
__attribute__((target("popcnt")))
#endif
size_t count_varints(const uint8_t* p, const uint8_t* end) {
    size_t n = 0;
    while (end - p >= 8) {
        uint64_t x;
        memcpy(&x, p, 8);
        n += (size_t)__builtin_popcountll(~x & 0x8080808080808080ull);
        p += 8;
    }
    while (p < end) n += !(*p++ & 0x80);
    return n;
}

// one varint, bounds-checked; false if truncated or longer than 10 bytes
inline bool varint_slow(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
    v = 0;
    for (int shift = 0; shift < 70; shift += 7) {
        if (p >= end) return false;
        const uint8_t b = *p++;
        v |= (uint64_t)(b & 0x7F) << shift;
        if (!(b & 0x80)) return true;
    }
    return false;
}

// the value of a varint of `len` <= 4 bytes held in the low bytes of y
inline uint64_t compact4(uint32_t y, int len) {
    const uint64_t v = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
    return v & ((1ull << (7 * len)) - 1);
}

bool decode_varints(const uint8_t* p, const uint8_t* end, int64_t* out, size_t n) {
    size_t i = 0;
    // two values per 8-byte load when both are short (the common case: ids of 1-4 bytes), which
    // halves the load -> length -> next-address dependency chain per value
    while (i + 2 <= n && end - p >= 8) {
        uint64_t x;
        memcpy(&x, p, 8);
        const uint64_t stops = ~x & 0x8080808080808080ull;
        const uint64_t s2 = stops & (stops - 1);
        const int e1 = stops ? __builtin_ctzll(stops) >> 3 : 8;  // terminator byte of value 1
        const int e2 = s2 ? __builtin_ctzll(s2) >> 3 : 8;        // terminator byte of value 2
        if (e1 < 4 && e2 - e1 <= 4 && e2 < 8) {
            out[i] = (int64_t)compact4((uint32_t)x, e1 + 1);
            out[i + 1] = (int64_t)compact4((uint32_t)(x >> (8 * (e1 + 1))), e2 - e1);
            i += 2;
            p += e2 + 1;
        } else if (e1 < 4) {
            out[i++] = (int64_t)compact4((uint32_t)x, e1 + 1);
            p += e1 + 1;
        } else {
            uint64_t v;
            if (!varint_slow(p, end, v)) return false;
            out[i++] = (int64_t)v;
        }
    }
    for (; i < n; ++i) {
        uint64_t v;
        if (!varint_slow(p, end, v)) return false;
        out[i] = (int64_t)v;
    }
    return p == end;
}

enum FeatureId { F_POS = 0, F_NEG = 1, F_W = 2, F_MODE = 3, F_NONE = -1 };
const char* const kNames[4] = {"positive_sample", "negative_sample", "subsampling_weight", "mode"};

FeatureId feature_id(const uint8_t* k, size_t n) {
    for (int i = 0; i < 4; ++i)
        if (strlen(kNames[i]) == n && !memcmp(kNames[i], k, n)) return (FeatureId)i;
    return F_NONE;
}

struct Parsed {
    std::vector<int64_t> i64[4];  // pos, neg, -, mode
    std::vector<float> w;
    void clear() {
        for (auto& v : i64) v.clear();
        w.clear();
    }
};

// Int64List / FloatList body -> values (packed or not). `want_float` selects the list kind that the
// VarLenFeature expects; the other kind is a type error as in tf.io.parse_single_example.
bool parse_list(Cursor c, bool want_float, std::vector<int64_t>& iv, std::vector<float>& fv) {
    while (c.more()) {
        const uint64_t tag = c.varint();
        const uint32_t field = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
        if (field != 1) {
            c.skip(wire);
            continue;
        }
        if (!want_float && wire == 0) {
            iv.push_back((int64_t)c.varint());
        } else if (!want_float && wire == 2) {
            Cursor s = c.sub();
            if (!s.ok) return false;
            const size_t n = count_varints(s.p, s.end), old = iv.size();
            iv.resize(old + n);
            if (!decode_varints(s.p, s.end, iv.data() + old, n)) return false;
        } else if (want_float && wire == 5) {
            float f;
            if ((size_t)(c.end - c.p) < 4) return false;
            memcpy(&f, c.p, 4);
            c.p += 4;
            fv.push_back(f);
        } else if (want_float && wire == 2) {
            Cursor s = c.sub();
            const size_t n = (size_t)(s.end - s.p);
            if (!s.ok || n % 4) return false;
            const size_t old = fv.size();
            fv.resize(old + n / 4);
            memcpy(fv.data() + old, s.p, n);
        } else {
            return false;
        }
    }
    return c.ok;
}

// Feature message -> the list of the expected kind. Returns false on a wrong kind.
bool parse_feature(Cursor c, FeatureId id, Parsed& out) {
    const bool want_float = id == F_W;
    std::vector<float> dummy_f;
    while (c.more()) {
        const uint64_t tag = c.varint();
        const uint32_t field = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
        if (wire != 2 || field < 1 || field > 3) {
            c.skip(wire);
            continue;
        }
        Cursor s = c.sub();
        if (!c.ok) return false;
        if (field == 1) return false;                       // bytes_list
        if ((field == 2) != want_float) return false;      // float vs int64 mismatch
        // protobuf merge semantics: a repeated oneof member appearing twice concatenates
        if (!parse_list(s, want_float, out.i64[id], want_float ? out.w : dummy_f)) return false;
    }
    return c.ok;
}

int parse_example(const uint8_t* data, size_t n, Parsed& out) {
    out.clear();
    Cursor ex{data, data + n};
    while (ex.more()) {
        const uint64_t tag = ex.varint();
        const uint32_t field = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
        if (field != 1 || wire != 2) {
            ex.skip(wire);
            continue;
        }
        Cursor feats = ex.sub();  // Features
        while (feats.more()) {
            const uint64_t t2 = feats.varint();
            if ((t2 >> 3) != 1 || (t2 & 7) != 2) {
                feats.skip((uint32_t)(t2 & 7));
                continue;
            }
            Cursor entry = feats.sub();  // map entry
            const uint8_t* key = nullptr;
            size_t klen = 0;
            Cursor val{nullptr, nullptr, false};
            while (entry.more()) {
                const uint64_t t3 = entry.varint();
                const uint32_t f3 = (uint32_t)(t3 >> 3), w3 = (uint32_t)(t3 & 7);
                if (w3 == 2 && (f3 == 1 || f3 == 2)) {
                    Cursor s = entry.sub();
                    if (f3 == 1) {
                        key = s.p;
                        klen = (size_t)(s.end - s.p);
                    } else {
                        val = s;
                    }
                } else {
                    entry.skip(w3);
                }
            }
            if (!entry.ok) return set_error(KGE_EINVAL, "tfrecord: malformed Features map entry");
            const FeatureId id = key ? feature_id(key, klen) : F_NONE;
            if (id == F_NONE || !val.ok) continue;
            if (!parse_feature(val, id, out))
                return set_error(KGE_EINVAL, "tfrecord: feature has the wrong list type or is malformed");
        }
        if (!feats.ok) return set_error(KGE_EINVAL, "tfrecord: malformed Features");
    }
    if (!ex.ok) return set_error(KGE_EINVAL, "tfrecord: malformed Example");
    return 0;
}

void put_varint(std::string& s, uint64_t v) {
    while (v >= 0x80) {
        s.push_back((char)(uint8_t)(v | 0x80));
        v >>= 7;
    }
    s.push_back((char)(uint8_t)v);
}

void put_tag(std::string& s, uint32_t field, uint32_t wire) { put_varint(s, ((uint64_t)field << 3) | wire); }

void put_bytes(std::string& s, uint32_t field, const std::string& body) {
    put_tag(s, field, 2);
    put_varint(s, body.size());
    s += body;
}

// Feature { int64_list | float_list { packed values } }
std::string feature_body(const int64_t* iv, const float* fv, int64_t n) {
    std::string packed;
    if (fv) {
        packed.assign((const char*)fv, (size_t)n * 4);
    } else {
        for (int64_t i = 0; i < n; ++i) put_varint(packed, (uint64_t)iv[i]);
    }
    std::string list;
    if (n > 0) put_bytes(list, 1, packed);  // proto3 omits an empty packed field
    std::string feat;
    put_bytes(feat, fv ? 2 : 3, list);
    return feat;
}

}  // namespace

struct kge_tfrecord_reader {
    std::vector<std::string> paths;
    size_t file = 0;
    FILE* fp = nullptr;
    int verify_crc = 1;
    std::vector<uint8_t> buf;
    Parsed rec;
    bool have = false;
};

struct kge_tfrecord_writer {
    FILE* fp = nullptr;
    std::string msg;
};

extern "C" {

uint32_t kge_crc32c(const void* data, int64_t n) { return crc32c((const uint8_t*)data, (size_t)(n > 0 ? n : 0)); }

kge_tfrecord_reader* kge_tfrecord_open(const char* const* paths, int64_t npaths, int verify_crc) {
    if (!paths || npaths <= 0) {
        set_error(KGE_EINVAL, "kge_tfrecord_open: no paths");
        return nullptr;
    }
    auto* r = new kge_tfrecord_reader();
    for (int64_t i = 0; i < npaths; ++i) {
        if (!paths[i]) {
            delete r;
            set_error(KGE_EINVAL, "kge_tfrecord_open: null path");
            return nullptr;
        }
        r->paths.emplace_back(paths[i]);
    }
    r->verify_crc = verify_crc;
    r->fp = fopen(r->paths[0].c_str(), "rb");
    if (!r->fp) {
        delete r;
        set_error(KGE_EINVAL, "kge_tfrecord_open: cannot open file");
        return nullptr;
    }
    return r;
}

void kge_tfrecord_close(kge_tfrecord_reader* r) {
    if (!r) return;
    if (r->fp) fclose(r->fp);
    delete r;
}

int kge_tfrecord_rewind(kge_tfrecord_reader* r) {
    if (!r) return set_error(KGE_EINVAL, "null reader");
    if (r->fp) fclose(r->fp);
    r->file = 0;
    r->have = false;
    r->fp = fopen(r->paths[0].c_str(), "rb");
    return r->fp ? 0 : set_error(KGE_EINVAL, "kge_tfrecord_rewind: cannot open file");
}

// Reads and parses the next Example (files in order, like TFRecordDataset(list)). Returns 1 and
// the element counts {positive_sample, negative_sample, subsampling_weight, mode} when a record was
// read, 0 at the end of the last file, or a negative error (truncated record, CRC mismatch, bad proto).
int kge_tfrecord_next(kge_tfrecord_reader* r, int64_t* counts) {
    if (!r || !counts) return set_error(KGE_EINVAL, "kge_tfrecord_next: bad arguments");
    r->have = false;
    for (;;) {
        if (!r->fp) return 0;
        uint8_t hdr[12];
        const size_t got = fread(hdr, 1, 12, r->fp);
        if (got == 0 && feof(r->fp)) {
            fclose(r->fp);
            r->fp = nullptr;
            if (++r->file >= r->paths.size()) return 0;
            r->fp = fopen(r->paths[r->file].c_str(), "rb");
            if (!r->fp) return set_error(KGE_EINVAL, "kge_tfrecord_next: cannot open file");
            continue;
        }
        if (got != 12) return set_error(KGE_EINVAL, "tfrecord: truncated record header");
        uint64_t len;
        uint32_t lcrc;
        memcpy(&len, hdr, 8);
        memcpy(&lcrc, hdr + 8, 4);
        if (r->verify_crc && lcrc != masked_crc(hdr, 8)) return set_error(KGE_EINVAL, "tfrecord: length CRC mismatch");
        if (len > ((uint64_t)1 << 40)) return set_error(KGE_EINVAL, "tfrecord: implausible record length");
        r->buf.resize((size_t)len + 4);
        if (fread(r->buf.data(), 1, (size_t)len + 4, r->fp) != (size_t)len + 4)
            return set_error(KGE_EINVAL, "tfrecord: truncated record");
        uint32_t dcrc;
        memcpy(&dcrc, r->buf.data() + len, 4);
        if (r->verify_crc && dcrc != masked_crc(r->buf.data(), (size_t)len))
            return set_error(KGE_EINVAL, "tfrecord: data CRC mismatch");
        const int rc = parse_example(r->buf.data(), (size_t)len, r->rec);
        if (rc) return rc;
        counts[0] = (int64_t)r->rec.i64[F_POS].size();
        counts[1] = (int64_t)r->rec.i64[F_NEG].size();
        counts[2] = (int64_t)r->rec.w.size();
        counts[3] = (int64_t)r->rec.i64[F_MODE].size();
        r->have = true;
        return 1;
    }
}

// Copies the last record's lists (sizes as returned by kge_tfrecord_next) into caller buffers.
int kge_tfrecord_copy(kge_tfrecord_reader* r, int64_t* positive_sample, int64_t* negative_sample,
                      float* subsampling_weight, int64_t* mode) {
    if (!r || !r->have) return set_error(KGE_EINVAL, "kge_tfrecord_copy: no record");
    const Parsed& p = r->rec;
    if ((!positive_sample && !p.i64[F_POS].empty()) || (!negative_sample && !p.i64[F_NEG].empty()) ||
        (!subsampling_weight && !p.w.empty()) || (!mode && !p.i64[F_MODE].empty()))
        return set_error(KGE_EINVAL, "kge_tfrecord_copy: null buffer");
    if (!p.i64[F_POS].empty()) memcpy(positive_sample, p.i64[F_POS].data(), p.i64[F_POS].size() * 8);
    if (!p.i64[F_NEG].empty()) memcpy(negative_sample, p.i64[F_NEG].data(), p.i64[F_NEG].size() * 8);
    if (!p.w.empty()) memcpy(subsampling_weight, p.w.data(), p.w.size() * 4);
    if (!p.i64[F_MODE].empty()) memcpy(mode, p.i64[F_MODE].data(), p.i64[F_MODE].size() * 8);
    return 0;
}

kge_tfrecord_writer* kge_tfrecord_writer_open(const char* path) {
    FILE* fp = path ? fopen(path, "wb") : nullptr;
    if (!fp) {
        set_error(KGE_EINVAL, "kge_tfrecord_writer_open: cannot create file");
        return nullptr;
    }
    auto* w = new kge_tfrecord_writer();
    w->fp = fp;
    return w;
}

// create_example + writer.write(example.SerializeToString()) (compress_data/utils.py:35-42,
// compress_data/main.py:117-131): one Example with the four lists, keys in sorted order.
int kge_tfrecord_write_example(kge_tfrecord_writer* w, const int64_t* positive_sample, int64_t npos,
                               const int64_t* negative_sample, int64_t nneg, const float* subsampling_weight,
                               int64_t nw, const int64_t* mode, int64_t nmode) {
    if (!w || !w->fp || npos < 0 || nneg < 0 || nw < 0 || nmode < 0 || (npos && !positive_sample) ||
        (nneg && !negative_sample) || (nw && !subsampling_weight) || (nmode && !mode))
        return set_error(KGE_EINVAL, "kge_tfrecord_write_example: bad arguments");
    // sorted keys: mode < negative_sample < positive_sample < subsampling_weight
    struct E {
        const char* key;
        std::string body;
    } entries[4] = {{"mode", feature_body(mode, nullptr, nmode)},
                    {"negative_sample", feature_body(negative_sample, nullptr, nneg)},
                    {"positive_sample", feature_body(positive_sample, nullptr, npos)},
                    {"subsampling_weight", feature_body(nullptr, subsampling_weight, nw)}};
    std::string feats;
    for (const E& e : entries) {
        std::string entry;
        put_bytes(entry, 1, e.key);
        put_bytes(entry, 2, e.body);
        put_bytes(feats, 1, entry);
    }
    std::string& ex = w->msg;
    ex.clear();
    put_bytes(ex, 1, feats);
    uint8_t hdr[12];
    const uint64_t len = ex.size();
    memcpy(hdr, &len, 8);
    const uint32_t lc = masked_crc(hdr, 8);
    memcpy(hdr + 8, &lc, 4);
    const uint32_t dc = masked_crc((const uint8_t*)ex.data(), ex.size());
    if (fwrite(hdr, 1, 12, w->fp) != 12 || fwrite(ex.data(), 1, ex.size(), w->fp) != ex.size() ||
        fwrite(&dc, 1, 4, w->fp) != 4)
        return set_error(KGE_EINVAL, "kge_tfrecord_write_example: write failed");
    return 0;
}

int kge_tfrecord_writer_close(kge_tfrecord_writer* w) {
    if (!w) return set_error(KGE_EINVAL, "null writer");
    const int rc = w->fp && fclose(w->fp) == 0 ? 0 : set_error(KGE_EINVAL, "kge_tfrecord_writer_close: close failed");
    delete w;
    return rc;
}

}  // extern "C"
