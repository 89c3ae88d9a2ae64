// report.cpp -- see report.h.
#include "report.h"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <string_view>
#include <unordered_map>

#include "fastq.h"

namespace fqhost {

HostAcc::HostAcc(int insert_size_max) : ism_(insert_size_max) {
    head_.assign((size_t)FQ_ACC_INSERT + (size_t)insert_size_max + 1, 0);
}

void HostAcc::add(const uint64_t* acc, int max_cycles) {
    for (size_t i = 0; i < head_.size(); ++i) head_[i] += acc[i];
    if (max_cycles > cap_) {
        for (auto& v : cyc_) v.resize((size_t)max_cycles * 16, 0);
        cap_ = max_cycles;
    }
    for (int k = 0; k < 4; ++k) {
        const uint64_t* st = acc + fq_acc_stats_offset(ism_, max_cycles, k);
        for (int f = 0; f < 4; ++f) st_[k][f] += st[f];
        const uint64_t* cy = st + FQ_ST_CYCLES;
        for (size_t i = 0; i < (size_t)max_cycles * 16; ++i) cyc_[k][i] += cy[i];
    }
    const uint64_t* t = acc + fq_acc_tail_offset(ism_, max_cycles);
    for (int j = 0; j < FQ_ACC_TAIL_WORDS; ++j) tail_[j] += t[j];
}

namespace {
uint64_t hash_bytes(const char* s, size_t n) {  // FNV-1a 64 over 8-byte words, then a final mix
    uint64_t h = 0xcbf29ce484222325ull ^ n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, s + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
    }
    uint64_t w = 0;
    if (i < n) std::memcpy(&w, s + i, n - i);
    h = (h ^ w) * 0x100000001b3ull;
    h ^= h >> 29;
    h *= 0xbf58476d1ce4e5b9ull;
    return h ^ (h >> 32);
}
}  // namespace

// one shard: open addressing over (hash, string) with the strings in a byte arena
struct AdapterCounts::Shard {
    struct Slot {
        uint64_t h = 0;
        uint64_t off = 0;
        uint32_t len = 0;
        uint32_t used = 0;
        size_t count = 0;
    };
    std::vector<Slot> slots = std::vector<Slot>(256);
    std::string arena;
    size_t n = 0;
    void bump(uint64_t h, const char* s, uint32_t len, size_t c) {
        size_t mask = slots.size() - 1, i = (h >> 6) & mask;
        for (;; i = (i + 1) & mask) {
            Slot& x = slots[i];
            if (!x.used) break;
            if (x.h == h && x.len == len && std::memcmp(arena.data() + x.off, s, len) == 0) {
                x.count += c;
                return;
            }
        }
        Slot& x = slots[i];
        x.used = 1;
        x.h = h;
        x.len = len;
        x.off = arena.size();
        x.count = c;
        arena.append(s, len);
        if (++n * 2 > slots.size()) grow();
    }
    void grow() {
        std::vector<Slot> old(slots.size() * 2);
        old.swap(slots);
        const size_t mask = slots.size() - 1;
        for (const Slot& x : old)
            if (x.used) {
                size_t i = (x.h >> 6) & mask;
                while (slots[i].used) i = (i + 1) & mask;
                slots[i] = x;
            }
    }
};

AdapterCounts::AdapterCounts() {
    for (int m = 0; m < 2; ++m)
        for (int k = 0; k < kShards; ++k) shards_[m].emplace_back(new Shard);
}
AdapterCounts::~AdapterCounts() = default;

void AdapterCounts::add(int mate, const std::string& a, size_t count) {
    const uint64_t h = hash_bytes(a.data(), a.size());
    shards_[mate][h % kShards]->bump(h, a.data(), (uint32_t)a.size(), count);
}

void AdapterCounts::add(const Pack& pk, const fq_read_result* res, const fq_params& p, Pool* pool) {
    const int mates = pk.paired ? 2 : 1;
    const int parts = pool ? std::max(1, std::min(pool->size() * 2, (pk.n + 16383) / 16384)) : 1;
    struct Item {
        uint64_t h;
        const char* s;
        uint32_t len;
    };
    // items[part][mate * kShards + shard]: the part's trimmed tails of that shard
    std::vector<std::vector<std::vector<Item>>> items((size_t)parts, std::vector<std::vector<Item>>((size_t)(2 * kShards)));
    auto hash_part = [&](int k) {
        const int i0 = (int)((int64_t)pk.n * k / parts), i1 = (int)((int64_t)pk.n * (k + 1) / parts);
        auto& it = items[(size_t)k];
        for (int i = i0; i < i1; ++i) {
            for (int m = 0; m < mates; ++m) {
                const fq_read_result& r = res[(size_t)i * mates + m];
                if (!(r.flags & (FQ_RF_AD_OVERLAP | FQ_RF_AD_SEQ)) || r.ad_len == 0) continue;
                const char* s = (r.flags & FQ_RF_AD_NEG)
                                    ? reinterpret_cast<const char*>(m ? p.adapter2 : p.adapter1) + r.ad_pos
                                    : pk.seq_text(m, (size_t)i) + r.ad_pos;
                const uint64_t h = hash_bytes(s, r.ad_len);
                it[(size_t)(m * kShards) + h % kShards].push_back(Item{h, s, r.ad_len});
            }
        }
    };
    auto merge_shard = [&](int j) {  // j = mate * kShards + shard
        Shard& sh = *shards_[j / kShards][(size_t)(j % kShards)];
        for (int k = 0; k < parts; ++k)
            for (const Item& x : items[(size_t)k][(size_t)j]) sh.bump(x.h, x.s, x.len, 1);
    };
    if (pool) {
        pool->run(parts, hash_part);
        pool->run(mates * kShards, merge_shard);
    } else {
        hash_part(0);
        for (int j = 0; j < mates * kShards; ++j) merge_shard(j);
    }
}

void AdapterCounts::add_entries(int m, const char* d, size_t bytes, const fq_params& p, Pool* pool) {
    const char* ad = reinterpret_cast<const char*>(m ? p.adapter2 : p.adapter1);
    auto next = [&](size_t o) { return o + (d[o + 2] ? 5 : 3 + ((uint8_t)d[o] | ((size_t)(uint8_t)d[o + 1] << 8))); };
    // ranges of 8192 entries (one pass over the lengths), hashed on the pool, then merged per shard
    std::vector<size_t> cuts{0};
    size_t k = 0;
    for (size_t o = 0; o + 3 <= bytes;) {
        o = next(o);
        if (++k % 8192 == 0 && o < bytes) cuts.push_back(o);
    }
    cuts.push_back(bytes);
    const int parts = (int)cuts.size() - 1;
    struct Item {
        uint64_t h;
        const char* s;
        uint32_t len;
    };
    std::vector<std::vector<std::vector<Item>>> items((size_t)parts, std::vector<std::vector<Item>>((size_t)kShards));
    auto hash_part = [&](int q) {
        auto& it = items[(size_t)q];
        for (size_t o = cuts[(size_t)q]; o + 3 <= cuts[(size_t)q + 1]; o = next(o)) {
            const uint32_t len = (uint8_t)d[o] | ((uint32_t)(uint8_t)d[o + 1] << 8);
            const char* s = d[o + 2] ? ad + ((uint8_t)d[o + 3] | ((uint32_t)(uint8_t)d[o + 4] << 8)) : d + o + 3;
            const uint64_t h = hash_bytes(s, len);
            it[h % kShards].push_back(Item{h, s, len});
        }
    };
    auto merge_shard = [&](int j) {
        Shard& sh = *shards_[m][(size_t)j];
        for (int q = 0; q < parts; ++q)
            for (const Item& x : items[(size_t)q][(size_t)j]) sh.bump(x.h, x.s, x.len, 1);
    };
    if (pool && parts > 1) {
        pool->run(parts, hash_part);
        pool->run(kShards, merge_shard);
    } else {
        for (int q = 0; q < parts; ++q) hash_part(q);
        for (int j = 0; j < kShards; ++j) merge_shard(j);
    }
}

AdapterCounts::Report AdapterCounts::report(int m) const {
    Report r;
    for (const auto& sh : shards_[m])
        for (const Shard::Slot& x : sh->slots)
            if (x.used) r.total += x.count;
    if (r.total == 0) return r;
    const double dt = (double)r.total;
    for (const auto& sh : shards_[m])
        for (const Shard::Slot& x : sh->slots)
            if (x.used && !(x.count / dt < 0.01)) r.top[sh->arena.substr(x.off, x.len)] = x.count;
    return r;
}

namespace {

}  // namespace

Summary summarize(const HostAcc& a, int k) {
    Summary s;
    s.reads = a.stat(k, FQ_ST_READS);
    s.length_sum = a.stat(k, FQ_ST_LENGTH_SUM);
    s.q20 = a.stat(k, FQ_ST_Q20);
    s.q30 = a.stat(k, FQ_ST_Q30);
    auto total_base = [&](int c) {
        uint64_t t = 0;
        for (int b = 0; b < 8; ++b) t += a.cyc(k, c, b);
        return t;
    };
    auto total_qual = [&](int c) {
        uint64_t t = 0;
        for (int b = 0; b < 8; ++b) t += a.cyc(k, c, 8 + b);
        return t;
    };
    int c = 0;
    for (c = 0; c < a.cycles_capacity(); ++c) {
        const uint64_t tb = total_base(c);
        s.bases += tb;
        if (tb == 0) break;
    }
    s.cycles = c;
    const int A = 'A' & 7, T = 'T' & 7, C = 'C' & 7, G = 'G' & 7, N = 'N' & 7;
    uint64_t content_g = 0, content_c = 0;
    for (int i = 0; i < s.cycles; ++i) {
        content_g += a.cyc(k, i, G);
        content_c += a.cyc(k, i, C);
    }
    s.gc = content_g + content_c;
    for (int b = 0; b < 8; ++b)
        for (int i = 0; i < s.cycles; ++i) s.base_contents[b] += a.cyc(k, i, b);
    Json qc = Json::object(), cc = Json::object();
    Json mean = Json::array();
    std::vector<double> meanv((size_t)s.cycles);
    for (int i = 0; i < s.cycles; ++i) {
        meanv[(size_t)i] = (double)total_qual(i) / (double)total_base(i);
        mean.push(Json::d(meanv[(size_t)i]));
    }
    s.qual_curves[4] = meanv;
    const char names[5] = {'A', 'T', 'C', 'G', 'N'};
    const int cls[5] = {A, T, C, G, N};
    for (int j = 0; j < 5; ++j) {
        Json qv = Json::array(), cv = Json::array();
        for (int i = 0; i < s.cycles; ++i) {
            const uint64_t cnt = a.cyc(k, i, cls[j]);
            const double q = cnt == 0 ? meanv[(size_t)i] : (double)a.cyc(k, i, 8 + cls[j]) / (double)cnt;
            const double c = (double)cnt / (double)total_base(i);
            if (j < 4) s.qual_curves[j].push_back(q);
            s.content_curves[j].push_back(c);
            qv.push(Json::d(q));
            cv.push(Json::d(c));
        }
        if (names[j] != 'N') qc[std::string(1, names[j])] = qv;
        cc[std::string(1, names[j])] = cv;
    }
    qc["Mean"] = mean;
    Json gcv = Json::array();
    for (int i = 0; i < s.cycles; ++i) {
        s.content_curves[5].push_back((double)(a.cyc(k, i, G) + a.cyc(k, i, C)) / (double)total_base(i));
        gcv.push(Json::d(s.content_curves[5].back()));
    }
    cc["GC"] = gcv;
    s.json["TotalReads"] = Json::u(s.reads);
    s.json["TotalBases"] = Json::u(s.bases);
    s.json["Q20Bases"] = Json::u(s.q20);
    s.json["Q30Bases"] = Json::u(s.q30);
    s.json["TotalCycles"] = Json::i(s.cycles);
    s.json["QualityCurves"] = qc;
    s.json["ContentCurves"] = cc;
    return s;
}

namespace {

// FilterResult::reportAdaptersJsonDetails, src/filterresult.cpp:231-251 (null when no adapters)
Json adapter_details(const AdapterCounts::Report& rep) {
    const size_t total = rep.total;
    Json j;
    if (total == 0) return j;
    const double dt = (double)total;
    size_t reported = 0;
    for (auto& e : rep.top) {
        if (e.second / dt < 0.01) continue;
        j[e.first] = Json::u(e.second);
        reported += e.second;
    }
    if (total - reported > 0) j["Others"] = Json::u(total - reported);
    return j;
}

}  // namespace

Json build_report(const Options& o, const HostAcc& a, const AdapterCounts& ac) {
    const bool paired = o.paired();
    Summary pre1 = summarize(a, 0), post1 = summarize(a, 2);
    Summary pre2, post2;
    if (paired) {
        pre2 = summarize(a, 1);
        post2 = summarize(a, 3);
    }
    // JsonReporter::report, src/jsonreporter.cpp:23-162
    long pre_reads = (long)(pre1.reads + pre2.reads), pre_bases = (long)(pre1.bases + pre2.bases);
    long pre_q20 = (long)(pre1.q20 + pre2.q20), pre_q30 = (long)(pre1.q30 + pre2.q30), pre_gc = (long)(pre1.gc + pre2.gc);
    long post_reads = (long)(post1.reads + post2.reads), post_bases = (long)(post1.bases + post2.bases);
    long post_q20 = (long)(post1.q20 + post2.q20), post_q30 = (long)(post1.q30 + post2.q30),
         post_gc = (long)(post1.gc + post2.gc);
    auto rate = [](long num, long den) { return den == 0 ? 0.0 : (double)num / den; };
    Json rep = Json::object();
    Json before = Json::object();
    before["TotalReads"] = Json::i(pre_reads);
    before["TotalBases"] = Json::i(pre_bases);
    before["Q20Bases"] = Json::i(pre_q20);
    before["Q30Bases"] = Json::i(pre_q30);
    before["Q20BaseRate"] = Json::d(rate(pre_q20, pre_bases));
    before["Q30BaseRate"] = Json::d(rate(pre_q30, pre_bases));
    before["Read1Length"] = Json::i(pre1.mean_length());
    if (paired) before["Read2Length"] = Json::i(pre2.mean_length());
    before["GCRate"] = Json::d(rate(pre_gc, pre_bases));
    rep["Summary"]["BeforeFiltering"] = before;
    Json after = Json::object();
    after["TotalReads"] = Json::i(post_reads);
    after["TotalBases"] = Json::i(post_bases);
    after["Q20Bases"] = Json::i(post_q20);
    after["Q30Bases"] = Json::i(post_q30);
    after["Q20BaseRate"] = Json::d(rate(post_q20, post_bases));
    after["Q30BaseRate"] = Json::d(rate(post_q30, post_bases));
    after["Read1Length"] = Json::i(post1.mean_length());
    if (paired) after["Read2Length"] = Json::i(post2.mean_length());
    after["GCRate"] = Json::d(rate(post_gc, post_bases));
    rep["Summary"]["AfterFiltering"] = after;

    Json fr = Json::object();  // FilterResult::reportJsonBasic, src/filterresult.cpp:204-222
    fr["PassedFilterReads"] = Json::u(a.filter(FQ_PASS_FILTER));
    fr["LowQualityReads"] = Json::u(a.filter(FQ_FAIL_QUALITY));
    fr["TooManyNReads"] = Json::u(a.filter(FQ_FAIL_N_BASE));
    if (o.correction) {
        fr["CorrectedReads"] = Json::u(a.tail(FQ_ACC_TAIL_CORRECTED_READS));
        fr["CorrectedBases"] = Json::u(a.tail(FQ_ACC_TAIL_CORRECTED_BASES));
    }
    if (o.complexity_filter) fr["LowComplexityReads"] = Json::u(a.filter(FQ_FAIL_COMPLEXITY));
    if (o.length_filter) {
        fr["TooShortReads"] = Json::u(a.filter(FQ_FAIL_LENGTH));
        if (o.max_len > 0) fr["TooLongReads"] = Json::u(a.filter(FQ_FAIL_TOO_LONG));
    }
    rep["FilterResult"] = fr;

    if (o.dup) {  // src/jsonreporter.cpp:99-108 with Duplicate::statAll's results
        Json d = Json::object();
        d["Rate"] = Json::d(a.dup_total == 0 ? 0.0 : (double)a.dup_dups / (double)a.dup_total);
        Json h = Json::array(), g = Json::array();
        for (int i = 0; i < o.dup_hist_size; ++i) {
            const uint64_t n = i < (int)a.dup_hist.size() ? a.dup_hist[(size_t)i] : 0;
            const uint64_t gs = i < (int)a.dup_gc_sum.size() ? a.dup_gc_sum[(size_t)i] : 0;
            h.push(Json::i((int32_t)n));
            g.push(Json::d((int)n > 0 ? (double)gs / 255.0 / (int)n : 0.0));
        }
        d["Histogram"] = h;
        d["MeanGC"] = g;
        rep["Duplication"] = d;
    }

    if (paired) {  // insert size, src/jsonreporter.cpp:107-114 + getPeakInsertSize src/peprocessor.cpp:249-259
        const int ism = a.insert_size_max();
        Json ins = Json::object();
        int peak = 0;
        long maxc = -1;
        Json hist = Json::array();
        for (int i = 0; i < ism; ++i) {
            const long v = (long)a.head()[FQ_ACC_INSERT + i];
            if (v > maxc) {
                peak = i;
                maxc = v;
            }
            hist.push(Json::i((int32_t)v));
        }
        ins["Peak"] = Json::i(peak);
        ins["Unknown"] = Json::i((long)a.head()[FQ_ACC_INSERT + ism]);
        ins["Histogram"] = hist;
        rep["InsertSize"] = ins;
    }

    if (o.adapter_trimming) {  // FilterResult::reportAdaptersJsonSummary, src/filterresult.cpp:296-318
        Json at = Json::object();
        at["AdapterTrimmedReads"] = Json::u(a.head()[FQ_ACC_ADAPTER_READS]);
        at["AdapterTrimmedBases"] = Json::u(a.head()[FQ_ACC_ADAPTER_BASES]);
        at["Read1AdapterSequence"] = Json::s(!o.adapter1.empty() ? o.adapter1 : o.detected_adapter1);
        if (paired) at["Read2AdapterSequence"] = Json::s(!o.adapter2.empty() ? o.adapter2 : o.detected_adapter2);
        at["Read1AdapterCounts"] = adapter_details(ac.report(0));
        if (paired) at["Read2AdapterCounts"] = adapter_details(ac.report(1));
        rep["AdapterTrim"] = at;
    }

    if (o.polyx || o.polyg) {  // FilterResult::reportPolyXTrimJson, src/filterresult.cpp:380-397
        Json px = Json::object();
        const char atcg[5] = {'A', 'T', 'C', 'G', 'N'};
        uint64_t rsum = 0, bsum = 0;
        Json pr = Json::object(), pb = Json::object();
        for (int b = 0; b < 5; ++b) {
            const uint64_t r = a.head()[FQ_ACC_POLYX_READS + b], bs = a.head()[FQ_ACC_POLYX_BASES + b];
            rsum += r;
            bsum += bs;
            pr[std::string(1, atcg[b])] = Json::u(r);
            pb[std::string(1, atcg[b])] = Json::u(bs);
        }
        // std::accumulate(..., 0) keeps an int: the totals wrap at 32 bits
        px["TotalPolyxTrimmedReads"] = Json::i((int32_t)(uint32_t)rsum);
        px["PolyxTrimmedReads"] = pr;
        px["TotalPolyxTrimmedBases"] = Json::i((int32_t)(uint32_t)bsum);
        px["PolyxTrimmedBases"] = pb;
        rep["PolyxTrimming"] = px;
    }
    rep["Read1BeforeFiltering"] = pre1.json;
    if (paired) rep["Read2BeforeFiltering"] = pre2.json;
    rep[o.merge ? "MergedAndFiltered" : "Read1AfterFiltering"] = post1.json;
    if (paired && !o.merge) rep["Read2AfterFiltering"] = post2.json;
    Json sw = Json::object();
    sw["CWD"] = Json::s(o.cwd);
    sw["Command"] = Json::s(o.command);
    sw["Version"] = Json::s(o.version);
    rep["Software"] = sw;
    return rep;
}

}  // namespace fqhost
