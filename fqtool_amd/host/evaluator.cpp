// evaluator.cpp -- the host pre-pass (reference src/evaluator.cpp, src/nucleotidetree.cpp):
// read-length estimate and paired-end adapter detection.  The detected adapter is only
// reported in the JSON (Read{1,2}AdapterSequence); trimming never uses it
// (src/filterresult.cpp:315-317).
#include "evaluator.h"

#include <fstream>
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>

#include "fastq.h"
#include "../../include/fqhost.h"

namespace fqhost {
namespace {

const char* const kKnownAdapters[] = {
#include "known_adapters.inc"
};

// Evaluator::int2seq, src/evaluator.cpp:49-59
std::string int2seq(size_t val, int len) {
    static const char bases[4] = {'A', 'T', 'C', 'G'};
    std::string s((size_t)len, 'N');
    for (int i = 0; i < len; ++i) {
        s[(size_t)(len - i - 1)] = bases[val & 3];
        val >>= 2;
    }
    return s;
}

// NucleotideTree::getDominantPath over the trie of a set of sequences (src/nucleotidetree.cpp:41-90),
// walked without building the trie: the path's node at depth d is reached by the sequences whose
// first d characters fall in the path's buckets (c & 7, NucleotideTree::addSeq stops at 'N').  At
// each node the children's counts are the next-character buckets of those sequences; the walk
// goes on while they total >= 50 and one bucket holds >= 95 % of them, and the node's base is the
// character of the first such sequence (in insertion order) that created it.  Each step keeps only
// the sequences that follow the dominant bucket, so the work is the path length times the
// surviving sequences, with no per-node allocation.
struct Seqs {  // sequence i = base[i][0 .. len[i]) read forward (dir 1) or backward (dir -1)
    std::vector<const char*> base;
    std::vector<int> len;
    int dir = 1;
    char at(size_t i, int d) const { return dir > 0 ? base[i][d] : base[i][-d]; }
};

std::string dominant_path(const Seqs& S, bool& reached_leaf) {
    std::string out;
    std::vector<uint32_t> live(S.base.size()), next;
    for (size_t i = 0; i < live.size(); ++i) live[i] = (uint32_t)i;
    for (int d = 0;; ++d) {
        int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        char first[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int total = 0;
        for (uint32_t i : live) {
            if (d >= S.len[i]) continue;
            const char c = S.at(i, d);
            if (c == 'N') continue;  // (addSeq stops at an uppercase N)
            const int b = c & 7;
            if (!cnt[b]) first[b] = c;
            ++cnt[b];
            ++total;
        }
        if (total < 50) break;
        int dom = -1;
        for (int b = 0; b < 8; ++b)
            if (cnt[b] && cnt[b] / (double)total >= 0.95) {
                dom = b;
                break;
            }
        if (dom < 0) {
            reached_leaf = false;
            break;
        }
        out += first[dom];
        next.clear();
        for (uint32_t i : live)
            if (d < S.len[i] && S.at(i, d) != 'N' && (S.at(i, d) & 7) == dom) next.push_back(i);
        live.swap(next);
    }
    return out;
}

// Evaluator::matchKnownAdapter, src/evaluator.cpp:428-446
std::string match_known(const std::string& seq) {
    for (const char* a : kKnownAdapters) {
        const size_t n = std::strlen(a);
        if (seq.size() < n) continue;
        if (seq.compare(0, n, a) == 0) return a;
    }
    return "";
}

// The detection pre-pass's reads: bases back to back, read i = seq[off[i] .. off[i + 1])
struct ReadSet {
    std::string seq;
    std::vector<uint32_t> off{0};
    size_t size() const { return off.size() - 1; }
};

// k-mer work on the GPU (fq_kmer_*, kmer.hip) unless a caller registered another backend
int gpu_open(int device, const uint8_t* seq, const uint32_t* off, int32_t n, void** out) {
    fq_kmer_set* k = nullptr;
    const int rc = fq_kmer_open(device, seq, off, n, &k);
    *out = k;
    return rc;
}
int gpu_close(void* h) { return fq_kmer_close(static_cast<fq_kmer_set*>(h)); }
int gpu_count(void* h, int32_t keylen, int32_t first, int32_t tail, uint32_t* counts) {
    return fq_kmer_count(static_cast<fq_kmer_set*>(h), keylen, first, tail, counts);
}
int gpu_find(void* h, int32_t keylen, int32_t first, int32_t tail, uint32_t seed, uint64_t* occ, size_t cap, size_t* n) {
    return fq_kmer_find(static_cast<fq_kmer_set*>(h), keylen, first, tail, seed, occ, cap, n);
}
const fqh_kmer_backend kGpuKmer = {gpu_open, gpu_close, gpu_count, gpu_find};
fqh_kmer_backend g_kmer = kGpuKmer;

// Evaluator::getAdapterWithSeed, src/evaluator.cpp:392-426: the occurrences of the seed come from
// the k-mer backend; the prefix trees do not depend on their order
std::string adapter_with_seed(int seed, const ReadSet& reads, void* kset, uint32_t seed_count, int keylen, int trim) {
    const int shift_tail = std::max(1, trim);
    std::vector<uint64_t> occ(seed_count);
    size_t n = 0;
    if (g_kmer.find(kset, keylen, 20, shift_tail, (uint32_t)seed, occ.data(), occ.size(), &n) != FQ_OK)
        throw std::runtime_error("adapter detection: k-mer search failed");
    n = std::min(n, occ.size());
    // the forward tree gets the read after the seed (minus the tail), the backward tree the read
    // before it, reversed (src/evaluator.cpp:405-414)
    Seqs fwd, bwd;
    fwd.base.reserve(n);
    fwd.len.reserve(n);
    bwd.base.reserve(n);
    bwd.len.reserve(n);
    bwd.dir = -1;
    for (size_t k = 0; k < n; ++k) {
        const size_t r = (size_t)(occ[k] >> 32);
        const int pos = (int)(uint32_t)occ[k];
        const char* s = reads.seq.data() + reads.off[r];
        const int len = (int)(reads.off[r + 1] - reads.off[r]);
        fwd.base.push_back(s + pos + keylen);
        fwd.len.push_back(len - keylen - shift_tail - pos);
        bwd.base.push_back(s + pos - 1);
        bwd.len.push_back(pos);
    }
    bool reached_leaf = true;
    const std::string f = dominant_path(fwd, reached_leaf);
    std::string b = dominant_path(bwd, reached_leaf);
    std::reverse(b.begin(), b.end());
    std::string adapter = b + int2seq((size_t)seed, keylen) + f;
    if (adapter.size() > 60) adapter.resize(60);
    const std::string known = match_known(adapter);
    if (!known.empty()) return known;
    return reached_leaf ? adapter : std::string();
}

}  // namespace

int evaluate_read_len(const std::string& path) {  // Evaluator::computeReadLen, src/evaluator.cpp:93-109
    FqReader r(path, false);
    std::string n, s, d, q;
    int len = 0;
    for (int i = 0; i < 1000 && r.read(n, s, d, q); ++i) len = std::max(len, (int)s.size());
    return len;
}

int evaluate_read_num(const std::string& path) {  // Evaluator::evaluateReadNum, src/evaluator.cpp:191-227
    const size_t kReadLimit = 512 * 1024, kBaseLimit = 151 * 512 * 1024;
    FqReader r(path, false, 1 << 20, true);
    ByteBuf text;
    Rec rec;
    size_t records = 0, bases = 0;
    uint64_t first_pos = 0;
    bool eof = false;
    while (records < kReadLimit && bases < kBaseLimit) {
        text.clear();
        if (!r.read(text, rec)) {
            if (!r.error().empty()) std::cerr << r.error();
            eof = true;
            break;
        }
        if (records == 0) first_pos = r.stream_pos();
        ++records;
        bases += rec.len;
    }
    if (eof) return (int)records;
    if (records <= 1) return 0;
    const uint64_t pos = r.stream_pos();
    std::ifstream is(path, std::ios::binary);  // bytesTotal: the file's size
    is.seekg(0, is.end);
    const double total = (double)(long long)is.tellg();
    const double per_read = (double)(pos - first_pos) / (double)(records - 1);
    return (int)(size_t)(total * 1.01 / per_read);
}

// Evaluator::evaluateAdapterSeq, src/evaluator.cpp:229-390
std::string detect_adapter(const std::string& path, int trim_tail1, std::string* msgs, int device) {
    const size_t kReadLimit = 256 * 1024, kBaseLimit = 151 * kReadLimit;
    // FQH_DETECT_TIMING=1: stage times on stderr (profiling aid, tools/detect_timing.py)
    static const bool timing = std::getenv("FQH_DETECT_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    std::string stages;
    auto stage = [&](const char* name) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        stages += std::string(" ") + name + " " + std::to_string(std::chrono::duration<double>(now - t_last).count());
        t_last = now;
    };
    struct Report {
        const std::string& s;
        const std::string& path;
        ~Report() {
            if (timing) std::cerr << "adapter detection " << path << ":" << s << std::endl;
        }
    } report{stages, path};
    FqReader r(path, false);
    ReadSet reads;
    size_t bases = 0;
    ByteBuf text;
    Rec rec;
    while (reads.size() < kReadLimit && bases < kBaseLimit) {
        text.clear();
        if (!r.read(text, rec)) {
            if (!r.error().empty()) {
                if (msgs) *msgs += r.error();
                else std::cerr << r.error();
            }
            break;
        }
        bases += rec.len;
        reads.seq.append(text.data() + rec.seq_off(), rec.len);
        reads.off.push_back((uint32_t)reads.seq.size());
    }
    stage("read");
    if (reads.size() < 10000) return "";
    const int shift_tail = std::max(1, trim_tail1);
    const int keylen = 10;
    const size_t size = (size_t)1 << (keylen * 2);
    // the 10-mer histogram of evaluateAdapterSeq (src/evaluator.cpp:265-279)
    void* kset = nullptr;
    if (g_kmer.open(device, reinterpret_cast<const uint8_t*>(reads.seq.data()), reads.off.data(), (int32_t)reads.size(),
                    &kset) != FQ_OK)
        throw std::runtime_error("adapter detection: no k-mer device (the pre-pass runs on the GPU)");
    struct Closer {
        void* h;
        ~Closer() { g_kmer.close(h); }
    } closer{kset};
    stage("open");
    std::vector<uint32_t> counts(size, 0);
    if (g_kmer.count(kset, keylen, 20, shift_tail, counts.data()) != FQ_OK)
        throw std::runtime_error("adapter detection: k-mer count failed");
    stage("count");
    counts[0] = 0;
    const int topnum = 10;
    int top[topnum] = {0};
    size_t total = 0;
    for (size_t k = 0; k < size; ++k) {
        int atcg[4] = {0, 0, 0, 0};
        for (int i = 0; i < keylen; ++i) ++atcg[(k >> (i * 2)) & 3];
        bool low = false;
        for (int b = 0; b < 4; ++b)
            if (atcg[b] >= keylen - 4) low = true;
        if (low) continue;
        if (atcg[2] + atcg[3] >= keylen - 2) continue;
        if ((k >> 12) == 0xff) continue;
        const size_t val = counts[k];
        total += val;
        for (int t = topnum - 1; t >= 0; --t) {
            if (val < counts[(size_t)top[t]]) {
                if (t < topnum - 1) {
                    for (int m = topnum - 1; m > t + 1; --m) top[m] = top[m - 1];
                    top[t + 1] = (int)k;
                }
                break;
            } else if (t == 0) {
                for (int m = topnum - 1; m > t; --m) top[m] = top[m - 1];
                top[t] = (int)k;
            }
        }
    }
    stage("top10");
    for (int t = 0; t < topnum; ++t) {
        const int key = top[t];
        if (key == 0) continue;
        const std::string sq = int2seq((size_t)key, keylen);
        const size_t count = counts[(size_t)key];
        if (count < 10 || count * size < total * 20) break;
        int diff = 0;
        for (size_t i = 0; i + 1 < sq.size(); ++i) diff += sq[i] != sq[i + 1];
        if (diff < 3) continue;
        const std::string est = adapter_with_seed(key, reads, kset, counts[(size_t)key], keylen, trim_tail1);
        stage("seed");
        if (!est.empty()) return est;
    }
    return "";
}

void set_kmer_backend(const fqh_kmer_backend* b) {
    if (b) g_kmer = *b;
    else g_kmer = kGpuKmer;
}

}  // namespace fqhost
