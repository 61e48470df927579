// kge_sampler.hip — host-side negative sampler of the training batches: the
// upstream KnowledgeGraphEmbedding `TrainDataset` (codes/dataloader.py, absent from the snapshot;
// its call sites are compress_data/main.py:64-73), re-implemented in C++ so that the negative
// sample ids are BIT-EXACT with the upstream numpy code for the same RNG state:
//
//   TrainDataset.__getitem__(idx):
//     head, relation, tail = triples[idx]
//     subsampling_weight = sqrt(1 / (count[(head, relation)] + count[(tail, -relation-1)]))   (start 4)
//     while size < N:
//       negative_sample = np.random.randint(nentity, size=2N)          # legacy MT19937, masked rejection
//       mask = np.in1d(negative_sample, true_head[(r, t)] or true_tail[(h, r)],
//                      assume_unique=True, invert=True)                # numpy 2.2 algorithm selection
//       keep negative_sample[mask]
//     negative_sample = concat(...)[:N]
//
// np.in1d (numpy 2.2.6 `_in1d`) picks one of three algorithms; two are exact membership tests, the
// third (sort with assume_unique=True) keeps only the LAST occurrence of a duplicated draw that is
// not a true triple. All three are reproduced. Host memory only; no GPU involved.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "kge_hip.h"

namespace kge_impl {
int set_error(int code, const char* msg);  // kge_abi.hip
}

namespace {

// MT19937 as numpy's legacy RandomState (mt19937_seed / mt19937_gen / mt19937_next32)
struct MT19937 {
    uint32_t key[624];
    int pos = 624;

    void seed(uint32_t s) {
        for (int i = 0; i < 624; ++i) {
            key[i] = s;
            s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
        }
        pos = 624;
    }
    void gen() {
        uint32_t y;
        int i;
        for (i = 0; i < 624 - 397; ++i) {
            y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
            key[i] = key[i + 397] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
        }
        for (; i < 623; ++i) {
            y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
            key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
        }
        y = (key[623] & 0x80000000u) | (key[0] & 0x7fffffffu);
        key[623] = key[396] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
        pos = 0;
    }
    static inline uint32_t temper(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    uint32_t next32() {
        if (pos >= 624) gen();
        return temper(key[pos++]);
    }
};

// numpy legacy RandomState.randint(high, size=n) for int64, high <= 2^32: masked rejection on 32-bit
// draws (random_bounded_uint64_fill, use_masked=True)
void randint(MT19937& mt, int64_t high, int64_t n, std::vector<int64_t>& out) {
    out.resize((size_t)n);
    const uint64_t rng = (uint64_t)(high - 1);
    if (rng == 0) {
        std::fill(out.begin(), out.end(), 0);
        return;
    }
    if (rng == 0xFFFFFFFFull) {
        for (int64_t i = 0; i < n; ++i) out[(size_t)i] = mt.next32();
        return;
    }
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    // branch-free rejection over whole MT blocks: every raw draw is consumed in order, an accepted one
    // advances k (the same draws, in the same order, as numpy's loop)
    const uint32_t lim = (uint32_t)rng;
    int64_t k = 0;
    while (k < n) {
        if (mt.pos >= 624) mt.gen();
        while (mt.pos < 624 && k < n) {
            const uint32_t v = MT19937::temper(mt.key[mt.pos++]) & mask;
            out[(size_t)k] = v;
            k += (v <= lim) ? 1 : 0;
        }
    }
}

struct TrueSet {
    std::vector<int64_t> ids;     // distinct, in insertion order (build) then sorted (finalize)
    int64_t lo = 0, hi = 0;

    // membership: most true sets hold a handful of ids, so a short linear scan beats hashing;
    // larger sets binary-search the sorted ids
    bool contains(int64_t v) const {
        if (v < lo || v > hi) return false;
        const size_t n = ids.size();
        if (n <= 16) {
            for (size_t i = 0; i < n; ++i)
                if (ids[i] == v) return true;
            return false;
        }
        return std::binary_search(ids.begin(), ids.end(), v);
    }
};

inline uint64_t pair_key(int64_t a, int64_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)(int32_t)b; }

}  // namespace

struct kge_sampler {
    std::vector<int64_t> triples;  // [T, 3]
    int64_t nentity = 0, nrelation = 0, nneg = 0;
    int mode = KGE_TAIL_BATCH;
    std::unordered_map<uint64_t, int64_t> count;  // (h, r) and (t, -r-1), start 4
    std::unordered_map<uint64_t, TrueSet> truth;  // (r, t) -> heads  or  (h, r) -> tails
    MT19937 mt;
    std::vector<int64_t> draw, kept;
    std::unordered_map<int64_t, int64_t> last;
};

namespace {

// appends ar1[np.in1d(ar1, ts.ids, assume_unique=True, invert=True)] to kept, as numpy 2.2.6 computes it
void append_kept(const std::vector<int64_t>& ar1, const TrueSet& ts, std::vector<int64_t>& kept,
                 std::unordered_map<int64_t, int64_t>& last) {
    const size_t n1 = ar1.size(), n2 = ts.ids.size();
    if (n2 == 0) {
        kept.insert(kept.end(), ar1.begin(), ar1.end());
        return;
    }
    const int64_t range = ts.hi - ts.lo;
    const bool table = range <= 6 * (int64_t)(n1 + n2);
    const bool loop = (double)n2 < 10.0 * pow((double)n1, 0.145);
    if (table || loop) {  // both are exact membership tests
        for (size_t i = 0; i < n1; ++i)
            if (!ts.contains(ar1[i])) kept.push_back(ar1[i]);
        return;
    }
    // stable mergesort path, assume_unique=True: a value not in ar2 survives only at its last index
    last.clear();
    for (size_t i = 0; i < n1; ++i) last[ar1[i]] = (int64_t)i;
    for (size_t i = 0; i < n1; ++i)
        if (!ts.contains(ar1[i]) && last[ar1[i]] == (int64_t)i) kept.push_back(ar1[i]);
}

}  // namespace

extern "C" {

kge_sampler* kge_sampler_create(const int64_t* triples, int64_t ntriples, int64_t nentity, int64_t nrelation,
                                int64_t negative_sample_size, int mode) {
    if (!triples || ntriples < 0 || nentity <= 0 || nrelation < 0 || negative_sample_size <= 0 ||
        (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH) || nentity > (int64_t)0xFFFFFFFF) {
        kge_impl::set_error(KGE_EINVAL, "kge_sampler_create: bad arguments");
        return nullptr;
    }
    kge_sampler* s = new kge_sampler();
    s->triples.assign(triples, triples + 3 * ntriples);
    s->nentity = nentity;
    s->nrelation = nrelation;
    s->nneg = negative_sample_size;
    s->mode = mode;
    for (int64_t i = 0; i < ntriples; ++i) {
        const int64_t h = triples[3 * i], r = triples[3 * i + 1], t = triples[3 * i + 2];
        // count_frequency(triples, start=4)
        for (uint64_t k : {pair_key(h, r), pair_key(t, -r - 1)}) {
            auto it = s->count.find(k);
            if (it == s->count.end())
                s->count.emplace(k, 4);
            else
                it->second += 1;
        }
        // get_true_head_and_tail: true_head[(r, t)] (head-batch) or true_tail[(h, r)] (tail-batch)
        const uint64_t k = mode == KGE_HEAD_BATCH ? pair_key(r, t) : pair_key(h, r);
        const int64_t v = mode == KGE_HEAD_BATCH ? h : t;
        TrueSet& ts = s->truth[k];
        if (ts.ids.empty()) ts.lo = ts.hi = v;
        ts.ids.push_back(v);
        ts.lo = std::min(ts.lo, v);
        ts.hi = std::max(ts.hi, v);
    }
    for (auto& kv : s->truth) {  // distinct, sorted
        auto& ids = kv.second.ids;
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    }
    s->mt.seed(0);
    return s;
}

void kge_sampler_destroy(kge_sampler* s) { delete s; }

int kge_sampler_seed(kge_sampler* s, uint32_t seed) {
    if (!s) return kge_impl::set_error(KGE_EINVAL, "null sampler");
    s->mt.seed(seed);
    return 0;
}

int kge_sampler_get(kge_sampler* s, const int64_t* idx, int64_t B, int64_t* pos_out, int64_t* neg_out,
                    float* weight_out) {
    if (!s || (B > 0 && (!idx || !pos_out || !neg_out || !weight_out)) || B < 0)
        return kge_impl::set_error(KGE_EINVAL, "kge_sampler_get: bad arguments");
    const int64_t T = (int64_t)(s->triples.size() / 3), N = s->nneg;
    static const TrueSet empty_set;
    for (int64_t b = 0; b < B; ++b) {
        const int64_t i = idx[b];
        if (i < 0 || i >= T) return kge_impl::set_error(KGE_EINVAL, "kge_sampler_get: index out of range");
        const int64_t h = s->triples[3 * i], r = s->triples[3 * i + 1], t = s->triples[3 * i + 2];
        pos_out[3 * b] = h;
        pos_out[3 * b + 1] = r;
        pos_out[3 * b + 2] = t;
        const int64_t c = s->count[pair_key(h, r)] + s->count[pair_key(t, -r - 1)];
        weight_out[b] = sqrtf(1.0f / (float)c);  // torch.sqrt(1 / torch.Tensor([c])) in fp32
        auto it = s->truth.find(s->mode == KGE_HEAD_BATCH ? pair_key(r, t) : pair_key(h, r));
        const TrueSet& ts = it == s->truth.end() ? empty_set : it->second;
        s->kept.clear();
        while ((int64_t)s->kept.size() < N) {
            randint(s->mt, s->nentity, 2 * N, s->draw);
            append_kept(s->draw, ts, s->kept, s->last);
        }
        memcpy(neg_out + b * N, s->kept.data(), (size_t)N * sizeof(int64_t));
    }
    return 0;
}

}  // extern "C"
