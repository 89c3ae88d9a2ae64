// evaluator.cpp -- the host pre-pass (reference src/evaluator.cpp, src/nucleotidetree.cpp):
// read-length estimate and paired-end adapter detection.  The detected adapter is only
// reported in the JSON (Read{1,2}AdapterSequence); trimming never uses it
// (src/filterresult.cpp:315-317).
#include "evaluator.h"

#include <fstream>
#include <algorithm>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>

#include "fastq.h"

namespace fqhost {
namespace {

const char* const kKnownAdapters[] = {
#include "known_adapters.inc"
};

// Evaluator::seq2int, src/evaluator.cpp:3-47
int seq2int(const std::string& seq, int pos, int keylen, int last) {
    auto code = [](char c) { return c == 'A' ? 0 : c == 'T' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : -1; };
    if (last >= 0) {
        const int mask = (1 << (keylen * 2)) - 1;
        const int b = code(seq[pos + keylen - 1]);
        if (b < 0) return -1;
        return ((last << 2) & mask) + b;
    }
    int key = 0;
    for (int i = pos; i < pos + keylen; ++i) {
        const int b = code(seq[i]);
        if (b < 0) return -1;
        key = (key << 2) + b;
    }
    return key;
}

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

// NucleotideTree, src/nucleotidetree.cpp:41-90
struct Node {
    int count = 0;
    char base = 'N';
    std::unique_ptr<Node> child[8];
};

void add_seq(Node* root, const std::string& s) {
    Node* cur = root;
    for (char c : s) {
        if (c == 'N') break;
        const int b = c & 7;
        if (!cur->child[b]) {
            cur->child[b].reset(new Node());
            cur->child[b]->base = c;
        }
        cur->child[b]->count++;
        cur = cur->child[b].get();
    }
}

std::string dominant_path(Node* root, bool& reached_leaf) {
    std::string out;
    Node* cur = root;
    for (;;) {
        int total = 0;
        for (int i = 0; i < 8; ++i)
            if (cur->child[i]) total += cur->child[i]->count;
        if (total < 50) break;
        bool dom = false;
        for (int i = 0; i < 8; ++i) {
            if (!cur->child[i]) continue;
            if (cur->child[i]->count / (double)total >= 0.95) {
                dom = true;
                out += cur->child[i]->base;
                cur = cur->child[i].get();
                break;
            }
        }
        if (!dom) {
            reached_leaf = false;
            break;
        }
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

// Evaluator::getAdapterWithSeed, src/evaluator.cpp:392-426
std::string adapter_with_seed(int seed, const std::vector<std::string>& reads, int keylen, int trim) {
    const int shift_tail = std::max(1, trim);
    Node fwd, bwd;
    for (const std::string& s : reads) {
        int key = -1;
        const int len = (int)s.size();
        for (int pos = 20; pos <= len - keylen - shift_tail; ++pos) {
            key = seq2int(s, pos, keylen, key);
            if (key == seed) {
                add_seq(&fwd, s.substr((size_t)(pos + keylen), (size_t)(len - keylen - shift_tail - pos)));
                std::string head = s.substr(0, (size_t)pos);
                std::reverse(head.begin(), head.end());
                add_seq(&bwd, head);
            }
        }
    }
    bool reached_leaf = true;
    const std::string f = dominant_path(&fwd, reached_leaf);
    std::string b = dominant_path(&bwd, reached_leaf);
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
std::string detect_adapter(const std::string& path, int trim_tail1, std::string* msgs) {
    const size_t kReadLimit = 256 * 1024, kBaseLimit = 151 * kReadLimit;
    FqReader r(path, false);
    std::vector<std::string> reads;
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
        reads.emplace_back(text.data() + rec.seq_off(), rec.len);
    }
    if (reads.size() < 10000) return "";
    const int shift_tail = std::max(1, trim_tail1);
    const int keylen = 10;
    const size_t size = (size_t)1 << (keylen * 2);
    std::vector<size_t> counts(size, 0);
    for (const std::string& sq : reads) {
        int key = -1;
        for (int pos = 20; pos <= (int)sq.size() - keylen - shift_tail; ++pos) {
            key = seq2int(sq, pos, keylen, key);
            if (key >= 0) ++counts[(size_t)key];
        }
    }
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
    for (int t = 0; t < topnum; ++t) {
        const int key = top[t];
        if (key == 0) continue;
        const std::string sq = int2seq((size_t)key, keylen);
        const size_t count = counts[(size_t)key];
        if (count < 10 || count * size < total * 20) break;
        int diff = 0;
        for (size_t i = 0; i + 1 < sq.size(); ++i) diff += sq[i] != sq[i + 1];
        if (diff < 3) continue;
        const std::string est = adapter_with_seed(key, reads, keylen, trim_tail1);
        if (!est.empty()) return est;
    }
    return "";
}

}  // namespace fqhost
