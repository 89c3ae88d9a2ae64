// fastq.cpp -- see fastq.h.
#include "fastq.h"
#include "pargz.h"

#include <algorithm>
#include <climits>
#include <cerrno>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <emmintrin.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <exception>
#include <future>
#include <iostream>
#include <memory>
#include <mutex>
#include <stdexcept>

namespace fqhost {

namespace {
constexpr int kBufSize = 1 << 20;  // src/fqreader.cpp:10

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

// first '\r' or '\n' in [p, p + n), or p + n
const char* line_end(const char* p, size_t n) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', n));
    const size_t upto = nl ? (size_t)(nl - p) : n;
    const char* cr = static_cast<const char*>(std::memchr(p, '\r', upto));
    return cr ? cr : p + upto;
}
std::mutex g_gate_mu;
std::shared_future<void> g_gate;  // invalid: no pre-pass running
}  // namespace

void set_reader_stderr_gate(std::shared_future<void> gate) {
    std::lock_guard<std::mutex> l(g_gate_mu);
    g_gate = std::move(gate);
}

void reader_stderr(const std::string& s) {
    if (s.empty()) return;
    std::shared_future<void> g;
    {
        std::lock_guard<std::mutex> l(g_gate_mu);
        g = g_gate;
    }
    if (g.valid()) g.wait();
    std::cerr << s << std::flush;
}

ByteBuf& ByteBuf::operator=(ByteBuf&& o) noexcept {
    if (this != &o) {
        release();
        p_ = o.p_;
        size_ = o.size_;
        cap_ = o.cap_;
        want_pinned_ = o.want_pinned_;
        is_pinned_ = o.is_pinned_;
        o.p_ = nullptr;
        o.size_ = o.cap_ = 0;
        o.is_pinned_ = false;
    }
    return *this;
}

extern std::atomic<uint64_t> g_pinned_bytes;

void ByteBuf::release() {
    if (!p_) return;
    if (is_pinned_) {
        fq_host_free(p_);
        g_pinned_bytes -= cap_;
    }
    else delete[] p_;
    p_ = nullptr;
    cap_ = size_ = 0;
    is_pinned_ = false;
}

std::atomic<uint64_t> g_pinned_regrows{0}, g_pinned_bytes{0};
static std::mutex g_retired_m;
// page-locked blocks outgrown mid-run: freed by the exit, or, for in-process callers of fqh_run, once
// no run is left whose copies might still target them (runs may overlap: a block retired by one run
// stays until every run that was active has ended)
static std::vector<std::pair<void*, size_t>> g_retired;
static size_t g_retired_bytes = 0;
static int g_pinned_runs = 0;

void pinned_run_begin() {
    std::lock_guard<std::mutex> g(g_retired_m);
    ++g_pinned_runs;
}

void pinned_run_end() {
    std::lock_guard<std::mutex> g(g_retired_m);
    if (--g_pinned_runs > 0) return;
    g_pinned_runs = 0;
    for (auto& b : g_retired) {
        fq_host_free(b.first);
        g_pinned_bytes -= b.second;
    }
    g_retired.clear();
    g_retired_bytes = 0;
}

void ByteBuf::reserve(size_t n) {
    if (n <= cap_) return;
    char* q = nullptr;
    bool pinned = false;
    if (want_pinned_) {
        // Page-locked buffers grow by at least 1/8 and to whole 2 MiB pages (fq_host_alloc maps
        // those anyway): a regrowth frees the old buffer, and unregistering page-locked memory
        // waits for the device to go idle, so a buffer that grows by a little for every slightly
        // larger window would stall the pipeline each time.
        if (is_pinned_) {
            n = std::max(n, cap_ + cap_ / 8);
            ++g_pinned_regrows;
        }
        retire_pinned_ = is_pinned_;  // (the old block is kept, see below)
        n = (n + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
        void* v = nullptr;
        if (fq_host_alloc(n, &v) == FQ_OK) {
            g_pinned_bytes += n;
            q = static_cast<char*>(v);
            pinned = true;
        } else {
            want_pinned_ = false;  // no device (CPU tests): ordinary memory from now on
        }
    }
    if (!q) q = new char[n];
    if (size_) std::memcpy(q, p_, size_);
    const size_t keep = size_;
    if (retire_pinned_ && is_pinned_) {
        // Unregistering page-locked memory waits for the device to go idle: a buffer that grows
        // mid-run (a pack's output, a staging window) leaves its old block registered until the
        // process ends instead of draining the pipeline here (up to 256 MiB of such blocks)
        std::lock_guard<std::mutex> g(g_retired_m);
        if (g_retired_bytes + cap_ <= ((size_t)256 << 20)) {
            g_retired.emplace_back(p_, cap_);
            g_retired_bytes += cap_;
            p_ = nullptr;
            cap_ = size_ = 0;
            is_pinned_ = false;
        }
    }
    retire_pinned_ = false;
    release();
    p_ = q;
    size_ = keep;
    cap_ = n;
    is_pinned_ = pinned;
}

FqReader::FqReader(const std::string& path, bool phred64, int buf_size, bool zlib_default_buffer)
    : phred64_(phred64), buf_size_(buf_size), buf_((size_t)buf_size) {
    if (ends_with(path, ".gz")) {
        gz_ = gzopen(path.c_str(), "r");
        if (!gz_) throw std::runtime_error("Failed to open file: " + path);
        if (!zlib_default_buffer) gzbuffer(gz_, 1 << 20);
        gzrewind(gz_);
    } else {
        fp_ = path == "/dev/stdin" ? stdin : std::fopen(path.c_str(), "rb");
        if (!fp_) throw std::runtime_error("Failed to open file: " + path);
    }
    fill();
}

uint64_t FqReader::stream_pos() const {
    if (gz_) return (uint64_t)gzoffset(gz_);
    const long t = std::ftell(fp_);
    return t < 0 ? 0 : (uint64_t)t;
}

FqReader::~FqReader() {
    if (gz_) gzclose(gz_);
    if (fp_ && fp_ != stdin) std::fclose(fp_);
}

void FqReader::fill() {  // FqReader::readToBuf, src/fqreader.cpp:30-44
    if (gz_) {
        len_ = gzread(gz_, buf_.data(), (unsigned)buf_size_);
        if (len_ < 0) {
            std::cerr << "Error to read gzip file" << std::endl;
            len_ = 0;
        }
        eof_ = gzeof(gz_) != 0 || len_ < buf_size_;
    } else {
        len_ = (int)std::fread(buf_.data(), 1, (size_t)buf_size_, fp_);
        eof_ = std::feof(fp_) != 0 || len_ < buf_size_;
    }
    used_ = 0;
}

// FqReader::getLine, src/fqreader.cpp:90-150: appends the next line to `out`.  A line ends at
// '\r' or '\n'; a '\n' right after the '\r' is consumed too unless the '\r' is the buffer's
// second-to-last byte or later (the reference's `end < len-1` test).
void FqReader::get_line(ByteBuf& out) {
    const int start = used_;
    const char* b = buf_.data();
    int end = start < len_ ? (int)(line_end(b + start, (size_t)(len_ - start)) - b) : start;
    if (end < len_ || len_ < buf_size_) {
        const int s = std::min(start, len_);
        const int k = std::max(0, end - start);
        if (k) std::memcpy(out.extend((size_t)k), b + s, (size_t)k);
        ++end;
        if (end < len_ - 1 && b[end] == '\n') ++end;
        used_ = end;
        return;
    }
    if (len_ > start) std::memcpy(out.extend((size_t)(len_ - start)), b + start, (size_t)(len_ - start));
    for (;;) {
        fill();
        b = buf_.data();
        end = len_ > 0 ? (int)(line_end(b, (size_t)len_) - b) : 0;
        if (end < len_ || len_ < buf_size_) {
            if (end) std::memcpy(out.extend((size_t)end), b, (size_t)end);
            ++end;
            if (end < len_ - 1 && b[end] == '\n') ++end;
            used_ = end;
            return;
        }
        if (len_) std::memcpy(out.extend((size_t)len_), b, (size_t)len_);
    }
}

// FqReader::read, src/fqreader.cpp:160-195
bool FqReader::read(ByteBuf& text, Rec& r) {
    err_.clear();
    if (used_ >= len_ && at_eof()) return false;
    const size_t off = text.size();
    get_line(text);
    for (;;) {  // skip to a line that starts with '@' (src/fqreader.cpp:169-171)
        const bool empty = text.size() == off;
        if ((empty && !(used_ >= len_ && at_eof())) || (!empty && text.data()[off] != '@')) {
            text.truncate(off);
            get_line(text);
        } else {
            break;
        }
    }
    if (text.size() == off) return false;
    const size_t name_len = text.size() - off;
    get_line(text);
    const size_t seq_len = text.size() - off - name_len;
    get_line(text);
    const size_t strand_len = text.size() - off - name_len - seq_len;
    get_line(text);
    const size_t qual_len = text.size() - off - name_len - seq_len - strand_len;
    char* p = text.data() + off;
    if (qual_len != seq_len) {
        const std::string name(p, name_len), seq(p + name_len, seq_len), strand(p + name_len + seq_len, strand_len),
            qual(p + name_len + seq_len + strand_len, qual_len);
        err_ = "Error: base sequnce and quality sequence have different length: \n" + name + "\n" + seq + "\n" + qual +
               "\n" + strand + "\n";
        text.truncate(off);
        return false;
    }
    if (phred64_) {  // Read::convertPhread64To33, src/read.h:71-75 (char arithmetic)
        char* q = p + name_len + seq_len + strand_len;
        for (size_t i = 0; i < qual_len; ++i) q[i] = (char)std::max(33, (int)q[i] - (64 - 33));
    }
    r.off = off;
    r.name_len = (uint32_t)name_len;
    r.strand_len = (uint32_t)strand_len;
    r.len = (uint32_t)seq_len;
    r.gap[0] = r.gap[1] = r.gap[2] = 0;
    return true;
}

bool FqReader::read(std::string& name, std::string& seq, std::string& strand, std::string& qual) {
    scratch_.clear();
    Rec r;
    if (!read(scratch_, r)) {
        if (!err_.empty()) std::cerr << err_;
        return false;
    }
    const char* p = scratch_.data();
    name.assign(p + r.off, r.name_len);
    seq.assign(p + r.seq_off(), r.len);
    strand.assign(p + r.strand_off(), r.strand_len);
    qual.assign(p + r.qual_off(), r.len);
    return true;
}

// ---- BGZF input ----
// A .gz regular file whose members all carry BGZF's 'BC' size field (bgzip, samtools, this tool's
// own writer) is inflated member by member on several threads: the member chain is walked from
// the headers alone when the file is opened (it must cover the file exactly), then batches of
// members are inflated in parallel into one buffer at their prefix-summed offsets, each checked
// against its CRC32 and ISIZE.  The byte stream is the one gzread would give; any other .gz goes
// through zlib's stream reader as in the reference (src/fqreader.cpp:3-16).
//
// Corrupt data: the reference reads gzip through gzread calls of `call` bytes (1 MiB,
// src/fqreader.cpp:28-35), and the call during which zlib meets the error returns -1, so the
// stream it sees ends at the start of that call: every earlier call's bytes, including the bad
// member's bytes that zlib had written out before its CRC / ISIZE check or its data error.  Here the
// bytes of a batch are handed out only up to the last call boundary before the batch's end until
// the next batch is known to be good, so the cut can fall anywhere before a bad member.
class BgzfSource {
   public:
    static std::unique_ptr<BgzfSource> open(const std::string& path, size_t call) {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return nullptr;
        struct stat st;
        if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 28) {
            ::close(fd);
            return nullptr;
        }
        void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) return nullptr;
        std::unique_ptr<BgzfSource> b(new BgzfSource(static_cast<const unsigned char*>(m), (size_t)st.st_size,
                                                     std::max<size_t>(call, 1)));
        if (!b->walk()) return nullptr;
        madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
        return b;
    }
    // up to `want` more bytes of the decompressed stream into dst; false on corrupt data, once the
    // bytes the reference's gzread calls would have returned before the failing one are handed out
    bool read(char* dst, size_t want, size_t& got) {
        got = 0;
        if (!started_) {
            started_ = true;
            fetch();
        }
        while (got < want) {
            if (q_.empty()) break;
            Batch& c = q_.front();
            if (pos_ == c.data.size()) {
                q_.pop_front();
                pos_ = 0;
                if (q_.empty() && !done_) fetch();
                continue;
            }
            const size_t at = c.base + pos_;
            if (at >= limit_) {
                if (done_) break;
                fetch();
                continue;
            }
            const size_t n = std::min(std::min(want - got, c.data.size() - pos_), limit_ - at);
            std::memcpy(dst + got, c.data.data() + pos_, n);
            pos_ += n;
            got += n;
        }
        // corrupt data: reported once, by the call that reaches the cut
        if (bad_ && !reported_) {
            while (!q_.empty() && pos_ == q_.front().data.size()) {
                q_.pop_front();
                pos_ = 0;
            }
            if (q_.empty() || q_.front().base + pos_ >= limit_) {
                reported_ = true;
                return false;
            }
        }
        return true;
    }
    ~BgzfSource() {
        if (ahead_.valid()) ahead_.wait();
        munmap(const_cast<unsigned char*>(map_), size_);
    }

   private:
    struct Member {
        size_t data, clen;  // deflate payload offset and length
        uint32_t crc, isize;
    };
    struct Batch {
        std::string data;  // inflated bytes of the batch's members (the bad one's as far as zlib got)
        size_t base = 0;   // stream offset of data[0]
        bool ok = true;
        size_t keep = 0;   // (!ok) stream offset where the reference's stream ends
        bool last = true;  // no member after the batch
    };
    BgzfSource(const unsigned char* m, size_t n, size_t call) : map_(m), size_(n), call_(call) {}
    static uint32_t le16(const unsigned char* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
    static uint32_t le32(const unsigned char* p) { return le16(p) | le16(p + 2) << 16; }
    // the member chain from the headers (RFC 1952 header, BGZF 'BC' extra subfield)
    bool walk() {
        for (size_t o = 0; o < size_;) {
            const unsigned char* h = map_ + o;
            if (size_ - o < 28 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4) || (h[3] & 0xe0)) return false;
            const size_t xlen = le16(h + 10);
            if (12 + xlen > size_ - o) return false;
            size_t bsize = 0;
            for (size_t x = 12; x + 4 <= 12 + xlen;) {
                const size_t slen = le16(h + x + 2);
                if (h[x] == 'B' && h[x + 1] == 'C' && slen == 2 && x + 6 <= 12 + xlen) bsize = le16(h + x + 4) + 1;
                x += 4 + slen;
            }
            size_t p = 12 + xlen;
            auto skipz = [&]() {
                while (o + p < size_ && h[p]) ++p;
                ++p;
            };
            if (h[3] & 8) skipz();   // FNAME
            if (h[3] & 16) skipz();  // FCOMMENT
            if (h[3] & 2) p += 2;    // FHCRC
            if (!bsize || bsize > size_ - o || p + 8 > bsize) return false;
            members_.push_back(Member{o + p, bsize - p - 8, le32(h + bsize - 8), le32(h + bsize - 4)});
            o += bsize;
        }
        return !members_.empty();
    }
    // the next batch (inflated now, or the one inflating ahead), queued behind the ones being read;
    // starts inflating the one after it.  Bytes go out up to the last call boundary before the end of
    // what is known to be good: a call is the reference's gzread, which fails as a whole.
    void fetch() {
        Batch b;
        if (ahead_.valid()) b = ahead_.get();
        else inflate_batch(b);
        if (!b.ok) {
            limit_ = b.keep;
            done_ = bad_ = true;
        } else if (b.last) {
            limit_ = b.base + b.data.size();
            done_ = true;
        } else {
            limit_ = (b.base + b.data.size()) / call_ * call_;
            ahead_ = std::async(std::launch::async, [this] {
                Batch n;
                inflate_batch(n);
                return n;
            });
        }
        q_.push_back(std::move(b));
    }
    // the members from next_member_ (~64 MB of output) inflated into b.data on up to kThreads
    // threads.  A member that fails its inflate, CRC32 or ISIZE check ends the stream: b.keep is
    // the start of the reference's gzread call that meets the failure (the bytes before it, the bad
    // member's included, are in b.data).
    void inflate_batch(Batch& b) {
        static const int kThreads = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2));
        const size_t first = next_member_;
        size_t end = first, total = 0;
        std::vector<size_t> at;
        // (FQ_BGZF_BATCH: a smaller batch, for the tests of cuts across batches)
        const char* be = getenv("FQ_BGZF_BATCH");
        const size_t kBatch = be && atoll(be) > 0 ? (size_t)atoll(be) : (size_t)64 << 20;
        while (end < members_.size() && (total < kBatch || end == first)) {
            at.push_back(total);
            total += members_[end].isize;
            ++end;
        }
        b.data.resize(total);
        b.base = stream_off_;
        const size_t cnt = end - first;
        next_member_ = end;
        stream_off_ += total;
        b.last = end >= members_.size();
        // bad: the lowest index (within the batch) of a member that failed, with how far zlib got
        // in it; each thread stops at its own first failure, enough since its later members could
        // only raise it
        std::atomic<size_t> bad{cnt};
        std::vector<size_t> fail_at(cnt + 1, 0);  // stream offset of the failing gzread byte
        const int nt = (int)std::min<size_t>((size_t)kThreads, cnt);
        auto fail = [&](size_t i, size_t where) {
            fail_at[i] = where;
            size_t cur = bad.load();
            while (i < cur && !bad.compare_exchange_weak(cur, i)) {
            }
        };
        auto work = [&](int t) {
            const size_t i0 = cnt * (size_t)t / nt, i1 = cnt * (size_t)(t + 1) / nt;
            z_stream z;
            std::memset(&z, 0, sizeof z);
            if (inflateInit2(&z, -15) != Z_OK) {
                fail(i0, b.base + at[i0]);
                return;
            }
            for (size_t i = i0; i < i1 && i < bad.load(); ++i) {
                const Member& mb = members_[first + i];
                inflateReset(&z);
                z.next_in = const_cast<Bytef*>(map_ + mb.data);
                z.avail_in = (uInt)mb.clen;
                Bytef* o = reinterpret_cast<Bytef*>(&b.data[0]) + at[i];
                unsigned char dummy;
                z.next_out = mb.isize ? o : &dummy;
                z.avail_out = mb.isize ? (uInt)mb.isize : 1u;
                const int rc = inflate(&z, Z_FINISH);
                if (rc != Z_STREAM_END) {
                    // a data error (or a member longer than its ISIZE): zlib fails while producing
                    // the byte after the ones it wrote
                    fail(i, b.base + at[i] + std::min<size_t>(z.total_out, mb.isize));
                    break;
                }
                if (z.total_out != mb.isize || (uint32_t)crc32(crc32(0, nullptr, 0), o, mb.isize) != mb.crc) {
                    // the trailer check fails after the member's last byte
                    fail(i, b.base + at[i] + (z.total_out ? z.total_out - 1 : 0));
                    break;
                }
            }
            inflateEnd(&z);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
        if (nt > 0) work(0);
        for (auto& x : th) x.join();
        const size_t bi = bad.load();
        if (bi == cnt) return;
        b.ok = false;
        b.last = true;
        next_member_ = members_.size();  // nothing after a bad member
        b.keep = fail_at[bi] / call_ * call_;  // the failing call's start
        // (the bytes of the members after the bad one are not part of the stream)
        const size_t inside = at[bi] + members_[first + bi].isize;
        if (b.data.size() > inside) b.data.resize(inside);
    }
    const unsigned char* map_;
    size_t size_;
    size_t call_;  // the reference's gzread request (its buffer size)
    std::vector<Member> members_;
    size_t next_member_ = 0;  // first member not yet inflated (or being inflated ahead)
    size_t stream_off_ = 0;   // stream offset of that member
    std::deque<Batch> q_;       // inflated batches in stream order; the front one is being read
    size_t pos_ = 0;            // bytes of q_.front() handed out
    size_t limit_ = 0;          // stream offset up to which bytes may go out
    bool started_ = false;
    bool done_ = false;         // no batch to fetch after the queued ones
    bool bad_ = false;          // ... because the stream is corrupt at limit_
    bool reported_ = false;     // read() has returned false for it
    std::future<Batch> ahead_;  // the next batch, inflating while the queued ones are read
};

// ---- whole gzip files through libdeflate ----
// A gzip file (one member or several, not BGZF) inflated at once with the system's libdeflate
// (loaded at run time; its C API is stable: alloc / gzip_decompress_ex / free) into an anonymous
// mapping, which the reader then parses like a mapped plain file (parallel parse, zero copy).
// libdeflate inflates about 2.5x faster than zlib's stream reader on FASTQ; the price is memory for
// the whole uncompressed text, so only inputs whose reserved output (kRatio x the compressed size)
// fits the budget take this path.  Any failure (no libdeflate, corrupt data, output larger than the
// reservation) leaves the file to zlib's stream reader from its start, which reproduces the
// reference's behaviour on corrupt input.
namespace {
}  // namespace
struct Libdeflate {
    void* (*alloc)();
    int (*gzip_ex)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
    int (*deflate_ex)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);  // raw deflate
    void (*free_)(void*);
    // compression (BGZF members): alloc_compressor(level), deflate_compress -> bytes or 0 if it did
    // not fit, free_compressor, crc32
    void* (*calloc_)(int);
    size_t (*compress)(void*, const void*, size_t, void*, size_t);
    void (*cfree)(void*);
    uint32_t (*crc32_)(uint32_t, const void*, size_t);
    bool ok = false, cok = false;
    Libdeflate() {
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = reinterpret_cast<void* (*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
        gzip_ex = reinterpret_cast<int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*)>(
            dlsym(h, "libdeflate_gzip_decompress_ex"));
        deflate_ex = reinterpret_cast<int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*)>(
            dlsym(h, "libdeflate_deflate_decompress_ex"));
        free_ = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_decompressor"));
        ok = alloc && gzip_ex && deflate_ex && free_;
        calloc_ = reinterpret_cast<void* (*)(int)>(dlsym(h, "libdeflate_alloc_compressor"));
        compress = reinterpret_cast<size_t (*)(void*, const void*, size_t, void*, size_t)>(dlsym(h, "libdeflate_deflate_compress"));
        cfree = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_compressor"));
        crc32_ = reinterpret_cast<uint32_t (*)(uint32_t, const void*, size_t)>(dlsym(h, "libdeflate_crc32"));
        const char* z = std::getenv("FQ_GZ_ZLIB");  // 1: BGZF members through zlib's deflate (A/B)
        cok = calloc_ && compress && cfree && crc32_ && !(z && std::string(z) == "1");
    }
};
const Libdeflate& libdeflate() {
    static const Libdeflate l;
    return l;
}
namespace {

// the inflated text of gzip file `path` in an anonymous mapping (*out, *n bytes; munmap the
// reserved *cap bytes), or false
bool inflate_whole(const std::string& path, char** out, size_t* n, size_t* cap) {
    const char* env = std::getenv("FQ_GZ_WHOLE");  // 0: always zlib's stream reader
    if (env && std::string(env) == "0") return false;
    const Libdeflate& ld = libdeflate();
    if (!ld.ok) return false;
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 18) {
        ::close(fd);
        return false;
    }
    const size_t csize = (size_t)st.st_size;
    void* cm = mmap(nullptr, csize, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (cm == MAP_FAILED) return false;
    madvise(cm, csize, MADV_SEQUENTIAL);
    constexpr size_t kRatio = 12;  // reservation per compressed byte (FASTQ inflates 3-5x)
    const size_t phys = (size_t)sysconf(_SC_PHYS_PAGES) * (size_t)sysconf(_SC_PAGE_SIZE);
    const size_t want = std::max<size_t>(csize * kRatio, 1 << 20);
    bool ok = want <= std::min(phys / 8, (size_t)32 << 30);  // (resident: only the bytes written)
    void* om = ok ? mmap(nullptr, want, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0)
                  : MAP_FAILED;
    ok = om != MAP_FAILED;
    size_t in = 0, outn = 0;
    if (ok) {
        madvise(om, want, MADV_HUGEPAGE);
        void* d = ld.alloc();
        ok = d != nullptr;
        while (ok && in < csize) {  // member by member
            size_t ain = 0, aout = 0;
            ok = ld.gzip_ex(d, static_cast<const char*>(cm) + in, csize - in, static_cast<char*>(om) + outn, want - outn,
                            &ain, &aout) == 0;
            in += ain;
            outn += aout;
            ok = ok && ain > 0;
        }
        if (d) ld.free_(d);
    }
    munmap(cm, csize);
    if (!ok) {
        if (om != MAP_FAILED) munmap(om, want);
        return false;
    }
    *out = static_cast<char*>(om);
    *n = outn;
    *cap = want;
    return true;
}
}  // namespace

// ---- single-stream gzip input ----
// zlib's stream reader (the reference's gzread, src/fqreader.cpp:28-35) on a thread of its own per
// input, running ahead of the parser: blocks of the inflated stream queue up (at most kAhead), so
// inflating overlaps parsing.  gzread is called with the reference's buffer size, so a corrupt
// member costs the same bytes as in the reference: those of the call that fails.
class GzAhead {
   public:
    GzAhead(gzFile gz, size_t call) : gz_(gz), call_(call), th_([this] { run(); }) {}
    ~GzAhead() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // up to want bytes of the stream into dst; false once the stream failed (after the bytes
    // before the failure were handed out)
    bool read(char* dst, size_t want, size_t& got) {
        got = 0;
        std::unique_lock<std::mutex> lk(m_);
        while (got < want) {
            cv_.wait(lk, [this] { return !q_.empty() || done_; });
            if (q_.empty()) return !bad_;
            std::string& b = q_.front();
            const size_t n = std::min(want - got, b.size() - off_);
            std::memcpy(dst + got, b.data() + off_, n);
            got += n;
            off_ += n;
            if (off_ == b.size()) {
                q_.pop_front();
                off_ = 0;
                cv_.notify_all();
            }
        }
        return true;
    }

   private:
    static constexpr size_t kBlock = 8u << 20;
    static constexpr size_t kAhead = 8;
    void run() {
        for (;;) {
            std::string b;
            const size_t cap = std::max(kBlock, call_);
            b.resize(cap);
            size_t n = 0;
            bool end = false, bad = false;
            while (n + call_ <= cap) {
                const int r = gzread(gz_, &b[n], (unsigned)call_);
                if (r < 0) {
                    bad = end = true;
                    break;
                }
                n += (size_t)r;
                if ((size_t)r < call_) {
                    end = true;
                    break;
                }
            }
            b.resize(n);
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [this] { return stop_ || q_.size() < kAhead; });
            if (stop_) return;
            if (n) q_.push_back(std::move(b));
            if (end) {
                done_ = true;
                bad_ = bad;
            }
            cv_.notify_all();
            if (end) return;
        }
    }
    gzFile gz_;
    size_t call_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::string> q_;
    size_t off_ = 0;
    bool stop_ = false, done_ = false, bad_ = false;
    std::thread th_;
};

// Half the host threads the process may use (its affinity, capped by OMP_NUM_THREADS), at least 2:
// the two mates of a pair inflate side by side.
int gz_inflate_threads() {
    if (const char* gt = std::getenv("FQ_GZ_THREADS"))  // (profiling: threads per file)
        if (std::atoi(gt) > 0) return std::atoi(gt);
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (const char* omp = std::getenv("OMP_NUM_THREADS"))
        if (std::atoi(omp) > 0) n = std::min(n, std::atoi(omp));
    return std::max(2, n / 2);
}

// ---- FqBulkReader ----
FqBulkReader::FqBulkReader(const std::string& path, bool phred64, int buf_size)
    : phred64_(phred64), bsize_((uint64_t)buf_size) {
    if (ends_with(path, ".gz")) {
        if ((bgzf_ = BgzfSource::open(path, (size_t)bsize_))) return;
        // a single-stream gzip file: chunks inflated on several threads
        if ((pargz_ = ParGzSource::open(path, (size_t)bsize_, gz_inflate_threads()))) return;
        path_ = path;
        // inflated whole on a thread of its own (so the mates of a pair inflate side by side), then
        // parsed like a mapped plain file; zlib's stream reader if that fails (settle())
        whole_ = std::async(std::launch::async, [path] {
            Whole w;
            w.ok = inflate_whole(path, &w.p, &w.n, &w.cap);
            return w;
        });
        return;
    }
    fp_ = path == "/dev/stdin" ? stdin : std::fopen(path.c_str(), "rb");
    if (!fp_) throw std::runtime_error("Failed to open file: " + path);
    struct stat st;
    if (fp_ != stdin && fstat(fileno(fp_), &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
        // a regular file is mapped (private, so phred64 conversion writes stay in this process).
        // Read-only unless phred64 rewrites it: the engine's text packs are copied to the GPU
        // straight from the mapping, and pinning writable private pages would copy them first.
        void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ | (phred64 ? PROT_WRITE : 0), MAP_PRIVATE, fileno(fp_), 0);
        if (m != MAP_FAILED) {
            madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
            map_ = static_cast<char*>(m);
            map_size_ = (size_t)st.st_size;
            total_ = map_size_;
            eof_ = true;
        }
    }
}

void FqBulkReader::settle() {
    if (!whole_.valid()) return;
    const Whole w = whole_.get();
    if (w.ok) {
        map_ = w.p;
        map_size_ = w.n;
        map_cap_ = w.cap;
        total_ = map_size_;
        eof_ = true;
        return;
    }
    gz_ = gzopen(path_.c_str(), "r");
    if (!gz_) throw std::runtime_error("Failed to open file: " + path_);
    gzrewind(gz_);  // (zlib's default buffer, as the reference: see FqReader)
    gz_ahead_.reset(new GzAhead(gz_, (size_t)bsize_));
}

FqBulkReader::~FqBulkReader() {
    if (whole_.valid()) {  // (never read: wait for the inflate, then unmap its output)
        const Whole w = whole_.get();
        if (w.ok) munmap(w.p, w.cap);
    }
    if (map_) munmap(map_, map_cap_ ? map_cap_ : map_size_);
    gz_ahead_.reset();  // (its thread reads gz_)
    if (gz_) gzclose(gz_);
    if (fp_ && fp_ != stdin) std::fclose(fp_);
}

void FqBulkReader::begin(ByteBuf& text) {
    settle();
    calls_ = 0;
    if (map_) {  // the mapping is the arena: offsets are file offsets, nothing is carried
        text.clear();
        text_ = nullptr;
        base_ = 0;
        tbase_ = pos_ >> 6;
        indexed_ = tbase_ << 6;
        return;
    }
    text_ = &text;
    text.clear();
    tbase_ = 0;
    indexed_ = 0;
    base_ = carry_off_;
    if (!carry_.empty()) std::memcpy(text.extend(carry_.size()), carry_.data(), carry_.size());
    carry_.clear();
    pos_ = 0;
}

const char* FqBulkReader::end() {
    if (map_) return map_;
    if (!text_) return nullptr;
    const size_t n = text_->size();
    if (pos_ < n) carry_.assign(text_->data() + pos_, n - pos_);
    else carry_.clear();
    carry_off_ = base_ + pos_;
    const char* base = text_->data();
    text_ = nullptr;
    return base;
}

// Reads up to the next buffer boundary past at least 4 MiB more (or to the end of the stream), so
// every reference buffer that holds an arena byte is complete in the arena.
void FqBulkReader::read_more() {
    const uint64_t want_end = (total_ + (4u << 20) + bsize_ - 1) / bsize_ * bsize_;
    size_t want = (size_t)(want_end - total_);
    char* dst = text_->extend(want);
    size_t got = 0;
    // (a failed source is reported when the parser first needs a byte past what it handed out --
    // where the reference's failing gzread call is made -- not here, ahead of the parser)
    if (bgzf_) {
        if (!bgzf_->read(dst, want, got)) src_failed_ = true;
    } else if (pargz_) {
        if (!pargz_->read(dst, want, got)) src_failed_ = true;
    } else if (gz_ahead_) {
        if (!gz_ahead_->read(dst, want, got)) src_failed_ = true;
    } else {
        got = std::fread(dst, 1, want, fp_);
    }
    text_->truncate(text_->size() - (want - got));
    total_ += got;
    if (got < want) {
        eof_ = true;
        pargz_.reset();  // (its workers are done: joined now, its buffers freed)
    }
}

// One SSE2 pass over new arena bytes: a bitmap of line terminators (word w of tidx_ covers arena
// bytes [64 (tbase_ + w), +64)), so finding the end of a line is a few word scans.
void FqBulkReader::index_to(size_t n) {
    const char* d = dat();
    const size_t w0 = indexed_ >> 6, w1 = (n + 63) >> 6;
    if (tidx_.size() < w1 - tbase_) tidx_.resize(w1 - tbase_ + 4096);
    const __m128i nl = _mm_set1_epi8('\n'), cr = _mm_set1_epi8('\r');
    for (size_t w = w0; w < w1; ++w) {
        const size_t base = w << 6;
        uint64_t m = 0;
        if (base + 64 <= n) {
            for (int k = 0; k < 4; ++k) {
                const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(d + base + 16 * k));
                const uint32_t mk =
                    (uint32_t)_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(v, nl), _mm_cmpeq_epi8(v, cr)));
                m |= (uint64_t)mk << (16 * k);
            }
        } else {
            for (size_t i = base; i < n; ++i)
                if (d[i] == '\n' || d[i] == '\r') m |= 1ull << (i - base);
        }
        tidx_[w - tbase_] = m;
    }
    indexed_ = n;
}

// first terminator in [x, n) (n <= indexed_), or n
size_t FqBulkReader::next_term(size_t x, size_t n) const {
    size_t w = x >> 6;
    uint64_t bits = tidx_[w - tbase_] & (~0ull << (x & 63));
    while (!bits) {
        if (((++w) << 6) >= n) return n;
        bits = tidx_[w - tbase_];
    }
    return std::min(n, (w << 6) + (size_t)__builtin_ctzll(bits));
}

// getLine's rule (src/fqreader.cpp:139-140): a '\n' right after a terminator at buffer index e is
// folded into it iff e + 1 < len - 1, len = that buffer's length (all but the stream's last
// buffer are full).
bool FqBulkReader::skip_ok(uint64_t g) const {
    const uint64_t k = g / bsize_, e = g - k * bsize_;
    const uint64_t len = (eof_ && total_ < (k + 1) * bsize_) ? total_ - k * bsize_ : bsize_;
    return e + 2 < len;
}

// the line at arena offset x: [x, e), next line at `next`; indexes (and reads) more of the stream
// as needed.  Past the end of the stream every line is empty (the reference's getLine at EOF).
bool FqBulkReader::line(size_t x, size_t& e, size_t& next) {
    for (;;) {
        const size_t n = sz();
        if (x < indexed_) {
            const size_t t = next_term(x, indexed_);
            if (t < indexed_) {
                const char* d = dat();
                e = t;
                next = t + 1;
                if (next < n && d[next] == '\n' && skip_ok(base_ + t)) ++next;
                return true;
            }
        }
        if (indexed_ < n) {  // index the next few MiB (the mapping is not indexed all at once)
            index_to(std::min(n, std::max(indexed_, x) + (4u << 20)));
            continue;
        }
        if (eof_) {  // the last line has no terminator, or we are past the end: empty lines
            demand_past_end();
            e = std::max(x, n);
            next = e + 1;
            return true;
        }
        read_more();
    }
}

bool FqBulkReader::read(Rec& r) {  // FqReader::read, src/fqreader.cpp:160-195
    err_.clear();
    ++calls_;
    if (at_end(pos_)) {  // (the reference's gzeof is still false here after a failed read: it reads)
        demand_past_end();
        return false;
    }
    size_t x = pos_, e = 0, nx = 0;
    line(x, e, nx);
    for (;;) {  // skip to a line that starts with '@' (src/fqreader.cpp:169-171)
        const bool empty = e == x;
        if ((empty && !at_end(nx)) || (!empty && dat()[x] != '@')) {
            x = nx;
            line(x, e, nx);
        } else {
            break;
        }
    }
    if (e == x) {
        pos_ = nx;
        return false;
    }
    const size_t name_off = x, name_len = e - x;
    size_t ls[3], le[3], ln[3];
    size_t y = nx;
    for (int k = 0; k < 3; ++k) {
        line(y, le[k], ln[k]);
        ls[k] = y;
        y = ln[k];
    }
    pos_ = y;
    const size_t seq_len = le[0] - ls[0], strand_len = le[1] - ls[1], qual_len = le[2] - ls[2];
    char* d = dat();
    if (qual_len != seq_len) {
        const size_t n = sz();
        auto str = [&](size_t a, size_t b) { return a < n ? std::string(d + a, std::min(b, n) - a) : std::string(); };
        err_ = "Error: base sequnce and quality sequence have different length: \n" + str(name_off, e) + "\n" +
               str(ls[0], le[0]) + "\n" + str(ls[2], le[2]) + "\n" + str(ls[1], le[1]) + "\n";
        return false;
    }
    if (phred64_) {  // Read::convertPhread64To33, src/read.h:71-75 (char arithmetic)
        char* q = d + ls[2];
        for (size_t i = 0; i < qual_len; ++i) q[i] = (char)std::max(33, (int)q[i] - (64 - 33));
    }
    r.off = name_off;
    r.name_len = (uint32_t)name_len;
    r.len = (uint32_t)seq_len;
    r.strand_len = (uint32_t)strand_len;
    r.gap[0] = (uint8_t)(ls[0] - e);
    r.gap[1] = (uint8_t)(ls[1] - le[0]);
    r.gap[2] = (uint8_t)(ls[2] - le[1]);
    return true;
}

// Parallel record location for a mapped file.  On a "plain" stretch -- every line ends in a single
// '\n', no line is empty (so no terminator is ever followed by a '\n' and getLine's 1 MiB-buffer
// folding rule, src/fqreader.cpp:139-140, never applies), every record's first line starts with
// '@' (so the skip loop of src/fqreader.cpp:169-171 never skips) and quality and sequence lengths
// agree (no error) -- FqReader::read is "four lines per record", which segments of the mapping can
// apply independently.  Segment k > 0 starts at its first line that looks like a record start ('@'
// line, a line, a '+' line, a line as long as the second); its records are kept only when segment
// k-1's parse ends exactly there (it started at a true record start, so its end is one), so a
// wrong guess is never used.  The fast path stops at the first segment it cannot take, or at the
// first irregular record, or where a record is not complete inside the region; read() continues
// from there with the exact rules.  Phred64 conversion is applied to the kept records only.
size_t FqBulkReader::read_fast(std::vector<Rec>& out, size_t max_n, Pool* pool) {
    if ((!map_ && !text_) || !pool || max_n < 1024) return 0;
    const size_t r0 = pos_, avg = avg_rec_ ? avg_rec_ : 512;
    const size_t want = r0 + max_n * avg + max_n * avg / 16 + (1u << 16);
    if (!map_)  // a stream (BGZF, gzip, pipe): the arena first holds the region, as far as the input goes
        while (!eof_ && sz() < want) read_more();
    if (pos_ >= sz()) return 0;
    char* d = dat();
    const size_t r1 = std::min(sz(), want);
    const size_t words = (r1 - r0 + 63) >> 6;
    std::vector<uint64_t> bm(words + 1, 0);  // bit i of word w: byte r0 + 64 w + i is '\r' / '\n'
    const int K = (int)std::max<size_t>(1, std::min<size_t>((size_t)pool->size() * 2, (r1 - r0) >> 20));
    const __m128i nl = _mm_set1_epi8('\n'), cr = _mm_set1_epi8('\r');
    pool->run(K, [&](int k) {
        const size_t w0 = words * k / K, w1 = words * (k + 1) / K;
        for (size_t w = w0; w < w1; ++w) {
            const size_t base = r0 + (w << 6);
            uint64_t m = 0;
            if (base + 64 <= r1) {
                for (int j = 0; j < 4; ++j) {
                    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(d + base + 16 * j));
                    m |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(v, nl), _mm_cmpeq_epi8(v, cr)))
                         << (16 * j);
                }
            } else {
                for (size_t i = base; i < r1; ++i)
                    if (d[i] == '\n' || d[i] == '\r') m |= 1ull << (i - base);
            }
            bm[w] = m;
        }
    });
    // first terminator at or after byte x (absolute), or r1
    auto term = [&](size_t x) -> size_t {
        if (x >= r1) return r1;
        size_t w = (x - r0) >> 6;
        uint64_t bits = bm[w] & (~0ull << ((x - r0) & 63));
        while (!bits) {
            if (++w >= words) return r1;
            bits = bm[w];
        }
        return std::min(r1, r0 + (w << 6) + (size_t)__builtin_ctzll(bits));
    };
    struct Seg {
        size_t start = SIZE_MAX, stop = SIZE_MAX;  // first record; where the parse ended
        bool clean = false;                        // ended at the segment's end (not at a problem)
        std::vector<Rec> recs;
    };
    std::vector<Seg> segs((size_t)K);
    auto bound = [&](int k) { return k >= K ? r1 : r0 + (r1 - r0) * (size_t)k / (size_t)K; };
    pool->run(K, [&](int k) {
        Seg& sg = segs[(size_t)k];
        size_t x;
        if (k == 0) {
            x = r0;
        } else {  // the first record-like line at or after the segment's start
            x = term(bound(k) - 1) + 1;
            for (int tries = 0;; ++tries) {
                if (tries == 16 || x >= bound(k + 1)) return;
                const size_t a = term(x), b = term(a + 1), c = term(b + 1), e = term(c + 1);
                if (e >= r1) return;
                if (d[x] == '@' && b + 1 < r1 && d[b + 1] == '+' && e - c == b - a) break;
                x = a + 1;
            }
        }
        sg.start = x;
        const size_t lim = bound(k + 1);
        sg.recs.reserve((lim - x) / avg + 16);
        while (x < lim) {
            const size_t t0 = term(x), t1 = term(t0 + 1), t2 = term(t1 + 1), t3 = term(t2 + 1);
            if (t3 >= r1 || d[x] != '@' || d[t0] != '\n' || d[t1] != '\n' || d[t2] != '\n' || d[t3] != '\n' ||
                t0 == x || t1 == t0 + 1 || t2 == t1 + 1 || t3 == t2 + 1 || t3 - t2 != t1 - t0)
                break;  // not plain (or incomplete in the region): the exact reader takes over here
            Rec r;
            r.off = x;
            r.name_len = (uint32_t)(t0 - x);
            r.len = (uint32_t)(t1 - t0 - 1);
            r.strand_len = (uint32_t)(t2 - t1 - 1);
            r.gap[0] = r.gap[1] = r.gap[2] = 1;
            sg.recs.push_back(r);
            x = t3 + 1;
        }
        sg.stop = x;
        sg.clean = x >= lim;
    });
    // stitch: segment k is taken while it starts where segment k-1 ended
    size_t x = r0, got = 0;
    std::vector<std::pair<int, size_t>> taken;  // (segment, records taken)
    for (int k = 0; k < K && got < max_n; ++k) {
        const Seg& sg = segs[(size_t)k];
        if (sg.start != x) break;
        const size_t take = std::min(sg.recs.size(), max_n - got);
        if (take) {
            taken.emplace_back(k, take);
            got += take;
            const Rec& last = sg.recs[take - 1];
            x = last.qual_off() + last.len + 1;
        }
        if (take < sg.recs.size() || !sg.clean) {
            if (take == sg.recs.size()) x = sg.stop;
            break;
        }
    }
    if (!got) return 0;
    const size_t o0 = out.size();
    out.resize(o0 + got);
    std::vector<size_t> at(taken.size());
    for (size_t i = 0, a = o0; i < taken.size(); ++i) {
        at[i] = a;
        a += taken[i].second;
    }
    pool->run((int)taken.size(), [&](int i) {
        const Seg& sg = segs[(size_t)taken[(size_t)i].first];
        const size_t cnt = taken[(size_t)i].second;
        std::memcpy(out.data() + at[(size_t)i], sg.recs.data(), cnt * sizeof(Rec));
        if (phred64_)  // Read::convertPhread64To33, src/read.h:71-75 (char arithmetic)
            for (size_t j = 0; j < cnt; ++j) {
                char* q = d + sg.recs[j].qual_off();
                for (uint32_t b = 0; b < sg.recs[j].len; ++b) q[b] = (char)std::max(33, (int)q[b] - (64 - 33));
            }
    });
    avg_rec_ = std::max<size_t>(16, (x - r0) / got);
    pos_ = x;
    tbase_ = pos_ >> 6;  // read() indexes afresh from here
    indexed_ = tbase_ << 6;
    calls_ += got;
    return got;
}

// The parser needs a byte past the end of what the source handed out: where the reference makes
// its failing gzread call (src/fqreader.cpp:28-33), if the source failed.  Noted once, with the
// index (in this arena) of the record being read; PackReader prints it in the reference's order.
void FqBulkReader::demand_past_end() {
    if (src_failed_ && !src_reported_) {
        src_reported_ = true;
        src_hit_ = (int64_t)calls_ - 1;
    }
}

int64_t FqBulkReader::take_source_error() {
    const int64_t h = src_hit_;
    src_hit_ = -1;
    return h;
}

// ---- Pool ----
struct Pool::Impl {
    struct Job {
        int n = 0;
        const std::function<void(int)>* fn = nullptr;
        std::atomic<int> next{0}, done{0};
        std::mutex em;
        std::exception_ptr err;  // the first exception of any index, rethrown by run()
    };
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::deque<std::shared_ptr<Job>> jobs;
    std::vector<std::thread> threads;
    bool stop = false;

    // runs indices of `j` until none are left; true when this call finished the job's last one
    static bool work(Job& j) {
        bool last = false;
        for (int i; (i = j.next.fetch_add(1)) < j.n;) {
            try {
                (*j.fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> g(j.em);
                if (!j.err) j.err = std::current_exception();
            }
            if (j.done.fetch_add(1) + 1 == j.n) last = true;
        }
        return last;
    }
    void loop() {
        std::unique_lock<std::mutex> l(m);
        for (;;) {
            cv.wait(l, [&] { return stop || !jobs.empty(); });
            if (stop) return;
            std::shared_ptr<Job> j = jobs.front();
            if (j->next.load() >= j->n) {  // every index taken: drop it and look again
                jobs.pop_front();
                continue;
            }
            l.unlock();
            const bool last = work(*j);
            l.lock();
            if (last) done_cv.notify_all();
        }
    }
};

Pool::Pool(int workers) : impl_(new Impl), workers_(std::max(0, workers)) {
    for (int i = 0; i < workers_; ++i) impl_->threads.emplace_back([this] { impl_->loop(); });
}

Pool::~Pool() {
    {
        std::lock_guard<std::mutex> l(impl_->m);
        impl_->stop = true;
    }
    impl_->cv.notify_all();
    for (auto& t : impl_->threads) t.join();
}

void Pool::run(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (workers_ == 0 || n == 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    auto j = std::make_shared<Impl::Job>();
    j->n = n;
    j->fn = &fn;
    {
        std::lock_guard<std::mutex> l(impl_->m);
        impl_->jobs.push_back(j);
    }
    impl_->cv.notify_all();
    Impl::work(*j);
    std::unique_lock<std::mutex> l(impl_->m);
    impl_->done_cv.wait(l, [&] { return j->done.load() == n; });
    for (auto it = impl_->jobs.begin(); it != impl_->jobs.end(); ++it)
        if (*it == j) {
            impl_->jobs.erase(it);
            break;
        }
    if (j->err) std::rethrow_exception(j->err);
}

// ---- Pack ----
void Pack::clear() {
    n = 0;
    raw = false;
    recs = false;
    zc = false;
    segs[0].clear();
    segs[1].clear();
    hold.reset();
    stage = -1;
    rout.results = nullptr;
    rout.rec[0] = rout.rec[1] = nullptr;
    stride = 0;
    base[0] = base[1] = nullptr;
    for (int m = 0; m < 2; ++m) {
        text[m].clear();
        rec[m].clear();
        seq[m].clear();
        qual[m].clear();
        len[m].clear();
    }
    fix.clear();
    fix_arena.clear();
    flags.clear();
    use_flags = false;
}

fq_batch Pack::batch() const {
    fq_batch b{};
    b.n = n;
    b.stride = stride;
    b.seq1 = reinterpret_cast<const uint8_t*>(seq[0].data());
    b.qual1 = reinterpret_cast<const uint8_t*>(qual[0].data());
    b.len1 = len[0].data();
    b.seq2 = paired ? reinterpret_cast<const uint8_t*>(seq[1].data()) : nullptr;
    b.qual2 = paired ? reinterpret_cast<const uint8_t*>(qual[1].data()) : nullptr;
    b.len2 = paired ? len[1].data() : nullptr;
    b.flags = use_flags ? flags.data() : nullptr;
    return b;
}

bool pack_text(Pack& pk, Pool* pool, bool merged) {
    const int mates = pk.paired ? 2 : 1;
    const size_t n = (size_t)pk.n;
    std::atomic<bool> ok{true};
    for (int m = 0; m < mates; ++m) {
        const std::vector<Rec>& R = pk.rec[m];
        pk.span[m] = pk.arena(m);
        pk.span_bytes[m] = 0;
        pk.max_len[m] = 0;
        if (!n) continue;
        const uint64_t a = R[0].off, b = R[n - 1].qual_off() + R[n - 1].len;
        if (b - a > 0xFFFFFFFFull) return false;
        pk.span[m] = pk.arena(m) + a;
        pk.span_bytes[m] = b - a;
        pk.trec[m].resize(n);
        pk.out_text[m].resize_uninit(b - a + 16);  // (fq_text_out: + the final terminator an input may lack)
    }
    for (int m = mates; m < 2; ++m) {
        pk.span[m] = nullptr;
        pk.span_bytes[m] = 0;
        pk.max_len[m] = 0;
    }
    if (merged && mates == 2 && n) pk.out_text[0].resize_uninit(pk.span_bytes[0] + pk.span_bytes[1] + 24 * n + 16);
    const int parts = pool ? std::max(1, std::min(pool->size() * 2, (int)((n + 16383) / 16384))) : 1;
    std::vector<int> mx((size_t)parts * 2, 0);
    auto work = [&](int k) {
        const size_t i0 = n * (size_t)k / (size_t)parts, i1 = n * (size_t)(k + 1) / (size_t)parts;
        for (int m = 0; m < mates; ++m) {
            const std::vector<Rec>& R = pk.rec[m];
            const uint64_t a = R[0].off;
            fq_text_rec* T = pk.trec[m].data();
            int mxl = 0;
            for (size_t i = i0; i < i1; ++i) {
                const Rec& r = R[i];
                if (r.len > 65535 || r.name_len > 65535 || r.strand_len > 65535) {
                    ok = false;
                    return;
                }
                T[i] = fq_text_rec{(uint32_t)(r.off - a), (uint32_t)(r.seq_off() - a), (uint32_t)(r.strand_off() - a),
                                   (uint32_t)(r.qual_off() - a), (uint16_t)r.name_len, (uint16_t)r.strand_len,
                                   (uint16_t)r.len, 0};
                mxl = std::max(mxl, (int)r.len);
            }
            mx[(size_t)(2 * k + m)] = mxl;
        }
    };
    if (pool && parts > 1) pool->run(parts, work);
    else if (n) work(0);
    if (!ok) return false;
    int maxlen = 0;
    for (int k = 0; k < parts; ++k)
        for (int m = 0; m < mates; ++m) {
            pk.max_len[m] = std::max(pk.max_len[m], mx[(size_t)(2 * k + m)]);
            maxlen = std::max(maxlen, mx[(size_t)(2 * k + m)]);
        }
    pk.stride = std::max(16, (maxlen + 15) & ~15);
    for (int m = 0; m < 2; ++m) pk.tout.text[m] = m < mates && n ? pk.out_text[m].data() : nullptr;
    pk.tout.bytes[0] = pk.tout.bytes[1] = 0;
    pk.text_mode = true;
    return true;
}

void pack_tiles(Pack& pk, Pool* pool) {
    pk.text_mode = false;
    const int mates = pk.paired ? 2 : 1;
    size_t maxlen = 0;
    for (int m = 0; m < mates; ++m) {
        pk.len[m].resize((size_t)pk.n);
        for (int i = 0; i < pk.n; ++i) {
            const uint32_t l = pk.rec[m][(size_t)i].len;
            if (l > 65535) throw std::runtime_error("read longer than 65535 bases");
            pk.len[m][(size_t)i] = (uint16_t)l;
            maxlen = std::max<size_t>(maxlen, l);
        }
    }
    pk.stride = (int)std::max<size_t>(16, (maxlen + 15) & ~(size_t)15);
    const size_t bytes = fq_batch_bytes(pk.n, pk.stride);
    const size_t tile_bytes = (size_t)FQ_TILE_READS * (size_t)pk.stride;
    for (int m = 0; m < mates; ++m) {
        pk.seq[m].resize_uninit(bytes);
        pk.qual[m].resize_uninit(bytes);
    }
    for (int m = mates; m < 2; ++m) {
        pk.seq[m].clear();
        pk.qual[m].clear();
        pk.len[m].clear();
    }
    const int tiles = (pk.n + FQ_TILE_READS - 1) / FQ_TILE_READS;
    const int parts = pool ? std::min(tiles, pool->size() * 4) : 1;
    auto work = [&](int part) {
        const int t0 = (int)((int64_t)tiles * part / parts), t1 = (int)((int64_t)tiles * (part + 1) / parts);
        for (int m = 0; m < mates; ++m) {
            char* sp = pk.seq[m].data();
            char* qp = pk.qual[m].data();
            for (int t = t0; t < t1; ++t) {
                std::memset(sp + (size_t)t * tile_bytes, 0, tile_bytes);
                std::memset(qp + (size_t)t * tile_bytes, 0, tile_bytes);
                const int i1 = std::min(pk.n, (t + 1) * FQ_TILE_READS);
                for (int i = t * FQ_TILE_READS; i < i1; ++i) {
                    const Rec& r = pk.rec[m][(size_t)i];
                    const char* s = pk.arena(m) + r.seq_off();
                    const char* q = pk.arena(m) + r.qual_off();
                    for (uint32_t j = 0; j < r.len; j += FQ_CHUNK) {
                        const size_t k = std::min<size_t>(FQ_CHUNK, r.len - j);
                        const size_t o = fq_batch_offset(pk.stride, i, (int32_t)j);
                        std::memcpy(sp + o, s + j, k);
                        std::memcpy(qp + o, q + j, k);
                    }
                }
            }
        }
    };
    if (pool) pool->run(parts, work);
    else if (tiles) work(0);
}

void FqBulkReader::seek(uint64_t off) {
    settle();
    if (!map_) {
        // a stream read from its start: its bytes up to `off` are read (in the usual buffer-aligned
        // steps) and dropped, the rest of the last step is carried into the first arena
        if (total_ != 0 || text_) throw std::runtime_error("FqBulkReader::seek on a stream already read");
        ByteBuf scratch;
        text_ = &scratch;
        uint64_t before = 0;
        while (!eof_ && total_ < off) {
            scratch.clear();
            before = total_;
            read_more();
        }
        text_ = nullptr;
        const uint64_t a = std::min<uint64_t>(std::max<uint64_t>(off, before), total_);
        carry_.assign(scratch.data() + (a - before), (size_t)(total_ - a));
        carry_off_ = a;
        return;
    }
    pos_ = (size_t)std::min<uint64_t>(off, map_size_);
    tbase_ = pos_ >> 6;
    indexed_ = tbase_ << 6;
}

// ---- PackReader ----
PackReader::PackReader(const std::string& in1, const std::string& in2, bool interleaved, bool phred64, int buf_size)
    : r1_(in1, phred64, buf_size), paired_(!in2.empty() || interleaved), interleaved_(interleaved) {
    if (!in2.empty() && !interleaved) r2_.reset(new FqBulkReader(in2, phred64, buf_size));
}

namespace {
size_t read_mate(FqBulkReader& r, Pack& pk, int m, size_t max_n, Pool* pool) {
    r.begin(pk.text[m]);
    Rec rc;
    pk.rec[m].reserve(max_n);
    size_t k = r.read_fast(pk.rec[m], max_n, pool);  // (mapped input: the plain stretch in parallel)
    while (k < max_n && r.read(rc)) {
        pk.rec[m].push_back(rc);
        ++k;
    }
    pk.base[m] = r.end();
    return k;
}
}  // namespace

void PackReader::seek(uint64_t off1, uint64_t off2, uint64_t first_seq) {
    r1_.seek(off1);
    if (r2_) r2_->seek(off2);
    packs_ = first_seq;
    done_ = false;
}

bool PackReader::next(Pack& pk, size_t max_n, Pool* pool) {
    if (done_) return false;
    const auto t0 = std::chrono::steady_clock::now();
    pk.clear();
    pk.paired = paired_;
    size_t n = 0;
    static const char* kGzErr = "Error to read gzip file\n";  // FqReader::readToBuf, src/fqreader.cpp:31-33
    if (!paired_) {
        n = read_mate(r1_, pk, 0, max_n, pool);
        if (r1_.take_source_error() >= 0) reader_stderr(kGzErr);
        if (n < max_n) {
            done_ = true;
            if (!r1_.error().empty()) reader_stderr(r1_.error());
        }
    } else if (interleaved_) {  // FqReaderPair over one file: mate 1, then mate 2
        r1_.begin(pk.text[0]);
        Rec a, b;
        while (n < max_n) {
            // FqReaderPair::read (src/fqreader.cpp:254-267) reads mate 2 even when mate 1 failed
            const bool ok_a = r1_.read(a);
            if (r1_.take_source_error() >= 0) reader_stderr(kGzErr);
            if (!ok_a) reader_stderr(r1_.error());
            const bool ok_b = r1_.read(b);
            if (r1_.take_source_error() >= 0) reader_stderr(kGzErr);
            if (!ok_a || !ok_b) {
                done_ = true;
                if (!ok_b) reader_stderr(r1_.error());
                break;
            }
            pk.rec[0].push_back(a);
            pk.rec[1].push_back(b);
            ++n;
        }
        pk.base[0] = pk.base[1] = r1_.end();
    } else {
        // One thread per mate.  FqReaderPair::read (src/fqreader.cpp:254-267) reads mate 1, then
        // mate 2 (always both), and stops once either failed: the pair count is the shorter run,
        // and a mate reports its error only if its failure is at that index (both do, read 1
        // first, when they fail at the same index).
        size_t n2 = 0;
        std::thread t([&] { n2 = read_mate(*r2_, pk, 1, max_n, pool); });
        const size_t n1 = read_mate(r1_, pk, 0, max_n, pool);
        t.join();
        n = std::min(n1, n2);
        // the messages in the reference's order: by pair index, mate 1 first, a gzip read error
        // before the same read's parse error; a mate's gzip error only if the reference got there
        struct Msg {
            size_t at;
            int mate, kind;
            const std::string* s;
        };
        static const std::string gz(kGzErr);
        std::vector<Msg> msgs;
        const int64_t h1 = r1_.take_source_error(), h2 = r2_->take_source_error();
        if (h1 >= 0 && (size_t)h1 <= n) msgs.push_back({(size_t)h1, 0, 0, &gz});
        if (h2 >= 0 && (size_t)h2 <= n) msgs.push_back({(size_t)h2, 1, 0, &gz});
        if (n < max_n) {
            done_ = true;
            if (n1 <= n2) msgs.push_back({n, 0, 1, &r1_.error()});
            if (n2 <= n1) msgs.push_back({n, 1, 1, &r2_->error()});
        }
        std::sort(msgs.begin(), msgs.end(), [](const Msg& a, const Msg& b) {
            return a.at != b.at ? a.at < b.at : a.mate != b.mate ? a.mate < b.mate : a.kind < b.kind;
        });
        for (const Msg& m : msgs) reader_stderr(*m.s);
        pk.rec[0].resize(n);
        pk.rec[1].resize(n);
    }
    if (n == 0) return false;
    pk.n = (int)n;
    const auto t1 = std::chrono::steady_clock::now();
    if (!defer_tiles) pack_tiles(pk, pool);
    parse_s += std::chrono::duration<double>(t1 - t0).count();
    tiles_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    pk.seq_no = packs_++;
    reads_ += (uint64_t)pk.n * (paired_ ? 2 : 1);
    return true;
}

// ---- Writer ----
Writer::Writer(const std::string& path, int level) : gzip_(ends_with(path, ".gz")), level_(level) {
    fp_ = std::fopen(path.c_str(), "wb");
    if (!fp_) throw std::runtime_error("cannot open " + path);
    struct stat st;
    positional_ = !gzip_ && fstat(fileno(fp_), &st) == 0 && S_ISREG(st.st_mode);
}

void Writer::write_at(uint64_t off, const char* p, size_t n) {
    const int fd = fileno(fp_);
    while (n) {
        const ssize_t w = ::pwrite(fd, p, n, (off_t)off);
        if (w < 0) {
            if (errno == EINTR) continue;
            throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
        }
        if (w == 0) throw std::runtime_error("write failed: no progress");
        p += w;
        n -= (size_t)w;
        off += (uint64_t)w;
    }
}

void Writer::write_segs_at(uint64_t off, const iovec* v, size_t n) {
    const int fd = fileno(fp_);
    std::vector<iovec> part;  // (a short write resumes inside a range)
    for (size_t i = 0; i < n;) {
        const size_t k = std::min<size_t>(n - i, (size_t)IOV_MAX);
        part.assign(v + i, v + i + k);
        i += k;
        iovec* q = part.data();
        size_t left = k;
        while (left && q->iov_len == 0) ++q, --left;
        while (left) {
            const ssize_t w = ::pwritev(fd, q, (int)left, (off_t)off);
            if (w < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
            }
            if (w == 0) throw std::runtime_error("write failed: no progress");
            off += (uint64_t)w;
            size_t got = (size_t)w;
            while (left && got >= q->iov_len) {
                got -= q->iov_len;
                ++q;
                --left;
            }
            if (left) {
                q->iov_base = static_cast<char*>(q->iov_base) + got;
                q->iov_len -= got;
            }
            while (left && q->iov_len == 0) ++q, --left;
        }
    }
}

namespace {
// `s` as BGZF members (blocked gzip, SAM/BAM spec 4.1: each member of at most 65280 input bytes
// carries its compressed size in a 'BC' extra field), so readers -- this tool's included -- can
// inflate the members on several threads; any gzip reader reads them as a plain multi-member
// stream.  (src/writer.cpp:36-47 writes one gzwrite stream at level -z; the decompressed text is
// what parity compares.)  An empty `s` gives one empty member.
// One member's deflate payload through libdeflate (a compressor per thread and level, kept for the
// thread's life); a member that does not fit BGZF's 64 KiB is stored (one stored deflate block).
void bgzf_append(std::string& out, const char* in, size_t n, uint32_t crc, const char* data, size_t clen) {
    const uint32_t bsize = (uint32_t)(clen + 25);
    const unsigned char hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                                   (unsigned char)(bsize & 0xff), (unsigned char)(bsize >> 8)};
    out.append(reinterpret_cast<const char*>(hdr), 18);
    out.append(data, clen);
    const unsigned char tr[8] = {(unsigned char)crc, (unsigned char)(crc >> 8), (unsigned char)(crc >> 16),
                                 (unsigned char)(crc >> 24), (unsigned char)n, (unsigned char)(n >> 8),
                                 (unsigned char)(n >> 16), (unsigned char)(n >> 24)};
    out.append(reinterpret_cast<const char*>(tr), 8);
    (void)in;
}
std::string gzip_member_libdeflate(const char* sp, size_t sn, int level) {
    constexpr size_t kIn = 0xff00;
    const Libdeflate& ld = libdeflate();
    struct Cache {
        void* c[13] = {};
        ~Cache() {
            for (void* p : c)
                if (p) libdeflate().cfree(p);
        }
    };
    static thread_local Cache cache;
    const int lvl = std::min(12, std::max(1, level));
    void*& c = cache.c[lvl];
    if (!c) c = ld.calloc_(lvl);
    if (!c) throw std::runtime_error("libdeflate_alloc_compressor failed");
    std::string out;
    out.reserve(sn / 3 + 64);
    char tmp[65536];
    size_t o = 0;
    do {
        const size_t n = std::min(kIn, sn - o);
        const char* in = sp + o;
        const uint32_t crc = ld.crc32_(0, in, n);
        size_t clen = ld.compress(c, in, n, tmp, 65536 - 26);
        if (clen == 0) {  // stored: BFINAL, BTYPE 00, LEN, NLEN, the bytes
            tmp[0] = 1;
            tmp[1] = (char)(n & 0xff);
            tmp[2] = (char)(n >> 8);
            tmp[3] = (char)(~n & 0xff);
            tmp[4] = (char)((~n >> 8) & 0xff);
            std::memcpy(tmp + 5, in, n);
            clen = n + 5;
        }
        bgzf_append(out, in, n, crc, tmp, clen);
        o += n;
    } while (o < sn);
    return out;
}
std::string gzip_member(const char* sp, size_t sn, int level);
std::string gzip_member(const std::string& s, int level) { return gzip_member(s.data(), s.size(), level); }
std::string gzip_member(const char* sp, size_t sn, int level) {
    if (libdeflate().cok) return gzip_member_libdeflate(sp, sn, level);
    constexpr size_t kIn = 0xff00;
    z_stream z;
    std::memset(&z, 0, sizeof z);
    if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
        throw std::runtime_error("deflateInit2 failed");
    std::string out;
    std::string tmp(deflateBound(&z, (uLong)kIn) + 64, '\0');
    int cur = level;
    size_t o = 0;
    do {
        const size_t n = std::min(kIn, sn - o);
        const Bytef* in = reinterpret_cast<const Bytef*>(sp + o);
        size_t clen = 0;
        for (int lvl : {level, 0}) {  // (a member that does not shrink enough is stored)
            deflateReset(&z);
            if (lvl != cur) {
                if (deflateParams(&z, lvl, Z_DEFAULT_STRATEGY) != Z_OK) throw std::runtime_error("deflateParams failed");
                cur = lvl;
            }
            z.next_in = const_cast<Bytef*>(in);
            z.avail_in = (uInt)n;
            z.next_out = reinterpret_cast<Bytef*>(&tmp[0]);
            z.avail_out = (uInt)tmp.size();
            if (deflate(&z, Z_FINISH) != Z_STREAM_END) throw std::runtime_error("deflate failed");
            clen = z.total_out;
            if (clen + 26 <= 65536) break;
        }
        if (clen + 26 > 65536) throw std::runtime_error("deflate: BGZF block too large");
        const uint32_t crc = (uint32_t)crc32(crc32(0, nullptr, 0), in, (uInt)n);
        bgzf_append(out, reinterpret_cast<const char*>(in), n, crc, tmp.data(), clen);
        o += n;
    } while (o < sn);
    deflateEnd(&z);
    return out;
}
}  // namespace

namespace {
void put(FILE* fp, const std::string& s) {
    if (!s.empty() && std::fwrite(s.data(), 1, s.size(), fp) != s.size())
        throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
}
}  // namespace

Writer::~Writer() {
    try {
        close();
    } catch (...) {  // a destructor cannot report; close() explicitly to see write errors
    }
}

void Writer::close() {
    if (!fp_) return;
    FILE* fp = fp_;
    fp_ = nullptr;
    try {
        if (gzip_ && !any_member_) put(fp, gzip_member(std::string(), level_));  // an empty .gz is one empty member
    } catch (...) {
        std::fclose(fp);
        throw;
    }
    if (std::fclose(fp) != 0) throw std::runtime_error(std::string("closing output failed: ") + std::strerror(errno));
}

void Writer::write_raw(const char* p, size_t n, Pool* pool) {
    if (!fp_) throw std::runtime_error("write to a closed output");
    if (!n) return;
    if (positional_) {
        write_at(claim(n), p, n);
        return;
    }
    if (!gzip_) {
        if (std::fwrite(p, 1, n, fp_) != n) throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
        return;
    }
    // one task of BGZF members per 1 MiB block on the pool, compressed from the caller's bytes, in
    // groups of 16 blocks: a group's members are written on a helper thread while the next group
    // compresses (the writes of one file are otherwise a serial gap in the pool's work)
    const size_t blk = (size_t)1 << 20;
    const int nb = (int)((n + blk - 1) / blk);
    constexpr int kGroup = 16;
    std::vector<std::string> z((size_t)nb);
    std::future<void> writing;
    for (int g0 = 0; g0 < nb; g0 += kGroup) {
        const int g1 = std::min(nb, g0 + kGroup);
        auto work = [&](int k) {
            const int i = g0 + k;
            const size_t o = (size_t)i * blk;
            z[(size_t)i] = gzip_member(p + o, std::min(blk, n - o), level_);
        };
        if (pool) pool->run(g1 - g0, work);
        else
            for (int k = 0; k < g1 - g0; ++k) work(k);
        if (writing.valid()) writing.get();  // (in order: the previous group first; rethrows its error)
        writing = std::async(std::launch::async, [this, &z, g0, g1] {
            for (int i = g0; i < g1; ++i)
                if (!z[(size_t)i].empty()) {
                    put(fp_, z[(size_t)i]);
                    std::string().swap(z[(size_t)i]);
                }
        });
        any_member_ = true;
    }
    if (writing.valid()) writing.get();
}

void Writer::write_segs(const iovec* v, size_t n) {
    if (!fp_) throw std::runtime_error("write to a closed output");
    if (gzip_) throw std::runtime_error("byte ranges go to plain outputs only");
    if (positional_) {
        size_t bytes = 0;
        for (size_t i = 0; i < n; ++i) bytes += v[i].iov_len;
        write_segs_at(claim(bytes), v, n);
        return;
    }
    if (std::fflush(fp_) != 0) throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
    const int fd = fileno(fp_);
    std::vector<iovec> part;  // (a short write resumes inside a range)
    for (size_t i = 0; i < n;) {
        const size_t k = std::min<size_t>(n - i, (size_t)IOV_MAX);
        part.assign(v + i, v + i + k);
        i += k;
        iovec* q = part.data();
        size_t left = k;
        while (left) {
            const ssize_t w = ::writev(fd, q, (int)left);
            if (w < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("write failed: ") + std::strerror(errno));
            }
            size_t got = (size_t)w;
            while (left && got >= q->iov_len) {
                got -= q->iov_len;
                ++q;
                --left;
            }
            if (left) {
                q->iov_base = static_cast<char*>(q->iov_base) + got;
                q->iov_len -= got;
            }
        }
    }
}

void Writer::write(const std::vector<std::string>& blocks, Pool* pool) {
    if (!fp_) throw std::runtime_error("write to a closed output");
    if (positional_) {
        for (const auto& s : blocks)
            if (!s.empty()) write_at(claim(s.size()), s.data(), s.size());
        return;
    }
    if (!gzip_) {
        for (const auto& s : blocks) put(fp_, s);
        return;
    }
    std::vector<std::string> z(blocks.size());
    auto work = [&](int i) {
        if (!blocks[(size_t)i].empty()) z[(size_t)i] = gzip_member(blocks[(size_t)i], level_);
    };
    if (pool) pool->run((int)blocks.size(), work);
    else
        for (int i = 0; i < (int)blocks.size(); ++i) work(i);
    for (const auto& s : z)
        if (!s.empty()) {
            put(fp_, s);
            any_member_ = true;
        }
}

}  // namespace fqhost
