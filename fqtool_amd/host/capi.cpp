// capi.cpp -- C entry points of the host library (libfqhost.so) for tests and bindings.
#include <cstdlib>
#include <fstream>
#include <memory>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "evaluator.h"
#include "json.h"
#include "options.h"
#include "pargz.h"
#include "processor.h"
#include "report.h"
#include "../../include/fqhost.h"

using namespace fqhost;

namespace {
int copy_out(const std::string& s, char* buf, size_t n) {
    if (!buf || n == 0) return -1;
    const size_t k = std::min(n - 1, s.size());
    std::memcpy(buf, s.data(), k);
    buf[k] = '\0';
    return (int)s.size();
}
}  // namespace

extern "C" {

int fqh_run(int argc, char** argv) { return run_tool(argc, argv); }

int fqh_json_double(double v, char* buf, size_t n) { return copy_out(json_double(v), buf, n); }

int fqh_merged_name(const char* name, int len1, int len2, char* buf, size_t n) {
    return copy_out(merged_name(name, len1, len2), buf, n);
}

int fqh_detect_adapter(const char* path, int trim_tail1, char* buf, size_t n) {
    try {
        return copy_out(detect_adapter(path, trim_tail1, nullptr, 0), buf, n);
    } catch (...) {
        return -1;
    }
}

int fqh_evaluate_read_len(const char* path) {
    try {
        return evaluate_read_len(path);
    } catch (...) {
        return -1;
    }
}

// JSON report from an accumulator block, for an argv (NUL-separated, argc entries) and adapter
// side information as text lines "D1\tSEQ" / "D2\tSEQ" (detected adapters) and
// "1\tSEQ\tCOUNT" / "2\tSEQ\tCOUNT" (adapter string counts).  Returns a malloc'd string.
char* fqh_report_json(int argc, const char* argv_blob, const uint64_t* acc, int max_cycles, const char* side) {
    try {
        std::vector<std::string> args;
        const char* p = argv_blob;
        for (int i = 0; i < argc; ++i) {
            args.emplace_back(p);
            p += args.back().size() + 1;
        }
        std::vector<char*> argv;
        for (auto& a : args) argv.push_back(&a[0]);
        Options o = parse_cli(argc, argv.data());
        o.update(argc, argv.data());
        AdapterCounts ac;
        std::istringstream in(side ? side : "");
        std::string line;
        while (std::getline(in, line)) {
            std::istringstream ls(line);
            std::string tag, seq;
            size_t cnt = 0;
            std::getline(ls, tag, '\t');
            std::getline(ls, seq, '\t');
            if (tag == "D1") o.detected_adapter1 = seq;
            else if (tag == "D2") o.detected_adapter2 = seq;
            else if (tag == "1" || tag == "2") {
                ls >> cnt;
                ac.add(tag == "1" ? 0 : 1, seq, cnt);
            }
        }
        HostAcc h(o.insert_size_max);
        h.add(acc, max_cycles);
        const std::string s = build_report(o, h, ac).dump(4);
        char* out = (char*)std::malloc(s.size() + 1);
        std::memcpy(out, s.c_str(), s.size() + 1);
        return out;
    } catch (const std::exception& e) {
        const std::string s = std::string("ERROR: ") + e.what();
        char* out = (char*)std::malloc(s.size() + 1);
        std::memcpy(out, s.c_str(), s.size() + 1);
        return out;
    }
}

void fqh_free(char* p) { std::free(p); }

void fqh_set_kmer_backend(const fqh_kmer_backend* b) { set_kmer_backend(b); }

// ---- host session: the tool's pipeline with the per-pack engine call left to the caller ----
struct fqh_session {
    Options o;
    std::unique_ptr<Pool> pool;  // -w threads: tile packing, formatting, gzip
    std::unique_ptr<PackReader> reader;
    Pack pk;
    std::unique_ptr<Sink> outs;
    HostAcc acc;
    AdapterCounts ac;
    std::string err;
    fqh_session() : acc(512) {}
};

const char* fqh_session_error(const fqh_session* s) { return s ? s->err.c_str() : ""; }

int fqh_session_open(int argc, char** argv, fqh_session** out) {
    std::unique_ptr<fqh_session> s(new fqh_session());
    try {
        s->o = prepare_options(argc, argv);
        s->acc = HostAcc(s->o.insert_size_max);
        s->reader.reset(new PackReader(s->o.in1, s->o.in2, s->o.interleaved, s->o.phred64));
        s->pool.reset(new Pool(std::max(0, s->o.threads - 1)));
        s->outs.reset(new Sink(s->o, s->pool.get()));
    } catch (const std::exception& e) {
        s->err = e.what();
        *out = s.release();
        return -1;
    }
    *out = s.release();
    return 0;
}

int fqh_session_params(fqh_session* s, int max_cycles, fq_params* out) {
    *out = s->o.to_params(max_cycles);
    return 0;
}

// next pack of up to max_n records; 1 = got one, 0 = end of input, -1 = error
int fqh_session_next(fqh_session* s, int max_n, fq_batch* out) {
    try {
        s->pk = Pack();
        if (!s->reader->next(s->pk, (size_t)max_n, s->pool.get())) return 0;
        prepare_pack(s->o, s->pk, s->pool.get());
        *out = s->pk.batch();
        return 1;
    } catch (const std::exception& e) {
        s->err = e.what();
        return -1;
    }
}

// formats the current pack from its per-read records, counts adapter strings and writes the
// output files like the tool
int fqh_session_consume(fqh_session* s, const fq_read_result* res, int max_cycles) {
    try {
        const fq_params p = s->o.to_params(max_cycles);
        apply_corrections(s->o, s->pk, res, s->pool.get());
        if (s->o.adapter_trimming) s->ac.add(s->pk, res, p);
        s->outs->consume(s->pk, res);
        return 0;
    } catch (const std::exception& e) {
        s->err = e.what();
        return -1;
    }
}

// -d: what the caller's duplication analysis needs, and its statAll result
int fqh_session_dup_params(fqh_session* s, int* enabled, int* keylen, int* hist_size) {
    *enabled = s->o.dup;
    *keylen = s->o.dup_keylen;
    *hist_size = s->o.dup_hist_size;
    return 0;
}

int fqh_session_set_dup(fqh_session* s, const uint64_t* hist, const uint64_t* gc_sum, const uint64_t* totals) {
    const size_t n = (size_t)s->o.dup_hist_size;
    s->acc.set_dup(std::vector<uint64_t>(hist, hist + n), std::vector<uint64_t>(gc_sum, gc_sum + n), totals[0], totals[1]);
    return 0;
}

int fqh_session_add_acc(fqh_session* s, const uint64_t* acc, int max_cycles) {
    s->acc.add(acc, max_cycles);
    return 0;
}

// closes the output files and writes the JSON report (-J); returns the report text
char* fqh_session_finish(fqh_session* s) {
    try {
        s->outs->close();
    } catch (const std::exception& e) {
        s->err = e.what();
        return nullptr;
    }
    const std::string t = build_report(s->o, s->acc, s->ac).dump(4);
    {
        std::ofstream js(s->o.json_file, std::ios::binary);
        js << t;
    }
    {
        std::ofstream hs(s->o.html_file, std::ios::binary);
        hs << build_html(s->o, s->acc, s->ac, html_time_now());
    }
    char* r = (char*)std::malloc(t.size() + 1);
    std::memcpy(r, t.c_str(), t.size() + 1);
    return r;
}

void fqh_session_close(fqh_session* s) { delete s; }

int fqh_pargz_read_all(const char* path, size_t call, int threads, size_t chunk, char** out, size_t* n, int* ok) {
    try {
        std::string s, how;
        bool good = true;
        if (!pargz_read_all(path, call, threads, chunk, s, good, how)) return 0;
        *out = static_cast<char*>(std::malloc(s.size() + 1));
        std::memcpy(*out, s.data(), s.size());
        *n = s.size();
        *ok = good ? 1 : 0;
        return how == "parallel" ? 1 : 2;
    } catch (...) {
        return -1;
    }
}

int fqh_gzread_all(const char* path, size_t call, char** out, size_t* n, int* ok) {
    gzFile g = gzopen(path, "r");  // (zlib's default buffer, as the reference's FqReader)
    if (!g) return -1;
    std::string s;
    std::vector<char> b(call);
    *ok = 1;
    for (;;) {  // as the reference's FqReader: a call that fails loses its bytes, a short one ends
        const int r = gzread(g, b.data(), (unsigned)call);
        if (r < 0) {
            *ok = 0;
            break;
        }
        s.append(b.data(), (size_t)r);
        if ((size_t)r < call) break;
    }
    gzclose(g);
    *out = static_cast<char*>(std::malloc(s.size() + 1));
    std::memcpy(*out, s.data(), s.size());
    *n = s.size();
    return 0;
}

int fqh_gz_drain(const char* path, size_t call, int threads, size_t chunk, size_t* n, int* ok, double* seconds) {
    try {
        std::vector<char> b(call);
        *n = 0;
        *ok = 1;
        const auto t0 = std::chrono::steady_clock::now();
        int rc = 0;
        if (threads > 0) {
            std::unique_ptr<ParGzSource> s = ParGzSource::open_chunked(path, call, threads, chunk);
            if (!s) return 0;
            for (;;) {
                size_t got = 0;
                const bool r = s->read(b.data(), call, got);
                *n += got;
                if (!r) *ok = 0;
                if (!r || got < call) break;
            }
            rc = s->fell_back() ? 2 : 1;
        } else {
            gzFile g = gzopen(path, "r");
            if (!g) return -1;
            for (;;) {
                const int r = gzread(g, b.data(), (unsigned)call);
                if (r < 0) *ok = 0;
                if (r <= 0) break;
                *n += (size_t)r;
                if ((size_t)r < call) break;
            }
            gzclose(g);
        }
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    } catch (...) {
        return -1;
    }
}

char* fqh_debug_records(const char* path, int bulk, int buf_size, int pack_n, int phred64) {
    std::string out;
    auto put = [&](const char* a, size_t la, const char* b, size_t lb, const char* c, size_t lc, const char* d,
                   size_t ld) {
        out.append(a, la).append("\t").append(b, lb).append("\t").append(c, lc).append("\t").append(d, ld).append("\n");
    };
    try {
        if (bulk) {  // 2: with the parallel fast path (read_fast on a 3-worker pool) ahead of read()
            FqBulkReader r(path, phred64 != 0, buf_size);
            ByteBuf text;
            Rec rc;
            std::vector<Rec> recs;
            std::unique_ptr<Pool> pool(bulk == 2 ? new Pool(3) : nullptr);
            for (bool more = true; more;) {
                r.begin(text);
                recs.clear();
                if (pool) r.read_fast(recs, (size_t)pack_n, pool.get());
                while ((int)recs.size() < pack_n && (more = r.read(rc))) recs.push_back(rc);
                const char* t = r.end();
                for (const Rec& x : recs)
                    put(t + x.off, x.name_len, t + x.seq_off(), x.len, t + x.strand_off(), x.strand_len, t + x.qual_off(),
                        x.len);
            }
            out += r.error();
        } else {
            FqReader r(path, phred64 != 0, buf_size);
            ByteBuf text;
            Rec rc;
            while (r.read(text, rc)) {
                const char* t = text.data();
                put(t + rc.off, rc.name_len, t + rc.seq_off(), rc.len, t + rc.strand_off(), rc.strand_len,
                    t + rc.qual_off(), rc.len);
                text.clear();
            }
            out += r.error();
        }
    } catch (const std::exception& e) {
        out += std::string("EXCEPTION: ") + e.what();
    }
    char* res = (char*)std::malloc(out.size() + 1);
    std::memcpy(res, out.c_str(), out.size() + 1);
    return res;
}

}  // extern "C"
