// fastq.h -- FASTQ input and output of the host tool.
//
// FqReader restates the reference reader (src/fqreader.cpp:3-195): 1 MiB buffered lines over
// zlib or stdio, a line ends at '\r' or '\n' ("\r\n" counts once, except at a buffer's last
// byte), records start at the next line beginning with '@', phred64 qualities are shifted at
// parse time (src/read.h:71-75) and a quality/sequence length mismatch ends the input
// (src/fqreader.cpp:184-191).  Unlike the reference it builds no std::string per field: records
// are appended to a pack's text arena and addressed by offsets.
//
// A Pack holds the records' text (per mate: name, seq, strand, qual back to back) and the
// engine's batch planes (chunk-interleaved tiles, include/fqengine.h), which pack_tiles fills
// from the text on a thread pool.  Writer restates src/writer.cpp (gzip level -z or plain).
#pragma once

#include <sys/uio.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fqengine.h"


namespace fqhost {

// The pack reader's stderr messages (record errors, gzip read errors) go through a gate: while the
// adapter-detection pre-pass runs concurrently with the pipeline (run_tool), they wait until the
// pre-pass has printed its own messages, so stderr keeps the reference's order (the reference
// runs the pre-pass first, src/main.cpp:139-143).
void set_reader_stderr_gate(std::shared_future<void> gate);
void reader_stderr(const std::string& s);
// page-locked blocks a run outgrew are kept registered until every run active with it has ended
void pinned_run_begin();
void pinned_run_end();

// Growable byte buffer that keeps its capacity when cleared (packs are recycled) and does not
// zero what it allocates.  A pinned buffer takes page-locked memory from the engine
// (fq_host_alloc: the H2D/D2H DMA then overlaps the kernels); without a HIP device it silently
// uses ordinary memory, which the engine also accepts (synchronous copies).
class ByteBuf {
   public:
    explicit ByteBuf(bool pinned = false) : want_pinned_(pinned) {}
    ~ByteBuf() { release(); }
    ByteBuf(const ByteBuf&) = delete;
    ByteBuf& operator=(const ByteBuf&) = delete;
    ByteBuf(ByteBuf&& o) noexcept { *this = std::move(o); }
    ByteBuf& operator=(ByteBuf&& o) noexcept;
    char* data() { return p_; }
    const char* data() const { return p_; }
    size_t size() const { return size_; }
    void clear() { size_ = 0; }
    void resize_uninit(size_t n) {
        reserve(n);
        size_ = n;
    }
    void reserve(size_t n);
    char* extend(size_t n) {  // appends n uninitialised bytes, returns their start
        if (size_ + n > cap_) reserve(std::max(size_ + n, cap_ + cap_ / 2 + 4096));
        char* r = p_ + size_;
        size_ += n;
        return r;
    }
    void truncate(size_t n) { size_ = n; }
    bool pinned() const { return is_pinned_; }

   private:
    void release();
    char* p_ = nullptr;
    size_t size_ = 0, cap_ = 0;
    bool want_pinned_ = false, is_pinned_ = false, retire_pinned_ = false;
};

// Array of T over a ByteBuf (read lengths, result records): pinned like its buffer.
template <class T>
class PodBuf {
   public:
    explicit PodBuf(bool pinned = false) : b_(pinned) {}
    void resize(size_t n) { b_.resize_uninit(n * sizeof(T)); }
    void clear() { b_.clear(); }
    size_t size() const { return b_.size() / sizeof(T); }
    T* data() { return reinterpret_cast<T*>(b_.data()); }
    const T* data() const { return reinterpret_cast<const T*>(b_.data()); }
    T& operator[](size_t i) { return data()[i]; }
    const T& operator[](size_t i) const { return data()[i]; }
    const T* begin() const { return data(); }
    const T* end() const { return data() + size(); }

   private:
    ByteBuf b_;
};

// One record's fields in a mate's text arena: name at off, then seq (len bytes), strand, qual,
// each field followed by gap[k] bytes of line terminator (0 when the fields were copied back to
// back; 1 or 2 -- "\r\n", or an empty line the reference's getLine folds into the terminator --
// when the arena holds the file's own bytes).
struct Rec {
    uint64_t off;
    uint32_t name_len, strand_len, len;
    uint8_t gap[3];
    size_t seq_off() const { return off + name_len + gap[0]; }
    size_t strand_off() const { return seq_off() + len + gap[1]; }
    size_t qual_off() const { return strand_off() + strand_len + gap[2]; }
};

class BgzfSource;
class ParGzSource;

class FqReader {
   public:
    // buf_size: the reference's read buffer (1 MiB, src/fqreader.cpp:10); smaller only in tests
    // zlib_default_buffer: keep zlib's own buffer size as the reference's reader does (the default):
    // a 1 MiB gzread then inflates straight into the caller's buffer, so a data or CRC error fails the
    // call whose bytes it lies in; with gzbuffer(1 MiB) zlib inflates 2 MiB ahead, and an error ends
    // the stream up to a call earlier (stream_pos() differs too)
    FqReader(const std::string& path, bool phred64, int buf_size = 1 << 20, bool zlib_default_buffer = true);
    ~FqReader();
    // FqReader::getBytes' bytesRead (src/fqreader.cpp:64-75): gzoffset / ftell of the stream
    uint64_t stream_pos() const;
    FqReader(const FqReader&) = delete;
    FqReader& operator=(const FqReader&) = delete;
    // Next record appended to `text`; false at end of input or on a quality/sequence length
    // mismatch, whose message (the reference's, src/fqreader.cpp:185-190) is left in error().
    bool read(ByteBuf& text, Rec& r);
    // Same, as strings (the evaluator pre-pass); prints a mismatch message like the reference.
    bool read(std::string& name, std::string& seq, std::string& strand, std::string& qual);
    const std::string& error() const { return err_; }

   private:
    void get_line(ByteBuf& out);
    void fill();
    bool at_eof() const { return eof_; }
    gzFile gz_ = nullptr;
    FILE* fp_ = nullptr;
    bool phred64_;
    int buf_size_;
    std::vector<char> buf_;
    int len_ = 0, used_ = 0;
    bool eof_ = false;
    std::string err_;
    ByteBuf scratch_;  // the string overload's record
};

// The pack reader's FqReader: same records, errors and line semantics as FqReader (and the
// reference), but zero copy: the file's bytes are read straight into the pack's text arena in
// large blocks and records are located in place (Rec with gaps).  getLine's treatment of a '\n'
// after a terminator depends on where the reference's 1 MiB read buffers end
// (src/fqreader.cpp:90-150), so reads stay aligned to buf_size multiples of the stream and the
// rule is evaluated on stream offsets.  Bytes read past the last record of a pack are carried
// into the next pack's arena.
class Pool;
class GzAhead;

// decoding threads of one single-stream gzip input (ParGzSource)
int gz_inflate_threads();

class FqBulkReader {
   public:
    FqBulkReader(const std::string& path, bool phred64, int buf_size = 1 << 20);
    ~FqBulkReader();
    FqBulkReader(const FqBulkReader&) = delete;
    FqBulkReader& operator=(const FqBulkReader&) = delete;
    // start filling `text` (cleared by the caller): the carried bytes go first
    void begin(ByteBuf& text);
    // next record into the arena given to begin(); false at end of input or on a
    // quality/sequence length mismatch (message in error())
    bool read(Rec& r);
    // Parallel fast path of read(): appends up to max_n records to `out` from the "plain" stretch
    // at the read position (see fastq.cpp) and returns their count; read() then continues exactly
    // where it stopped.  A mapped file is parsed in place; a stream (BGZF, gzip, pipe) once the
    // arena holds the region.
    size_t read_fast(std::vector<Rec>& out, size_t max_n, Pool* pool);
    // the arena is done: unconsumed bytes are carried to the next begin(); returns the base
    // the records' offsets refer to (the arena, or the file mapping)
    const char* end();
    const std::string& error() const { return err_; }
    // the index (read calls since begin()) at which the parser first needed bytes past a failed
    // gzip source -- the reference's "Error to read gzip file" -- or -1; cleared by the call
    int64_t take_source_error();
    bool mapped() {
        settle();
        return map_ != nullptr;
    }
    // the next record is read from stream offset off (a mapped file; or a stream not read yet,
    // whose bytes before off are then read and dropped)
    void seek(uint64_t off);
    bool parallel_gz() const { return pargz_ != nullptr; }  // a single-stream gzip file (ParGzSource)

   private:
    bool line(size_t x, size_t& e, size_t& next);
    void index_to(size_t n);                 // terminator bitmap of arena bytes [indexed_, n)
    size_t next_term(size_t x, size_t n) const;  // first '\r' / '\n' at or after x, or n
    bool at_end(size_t x) const { return eof_ && x >= sz(); }
    char* dat() const { return map_ ? map_ : text_->data(); }
    size_t sz() const { return map_ ? map_size_ : text_->size(); }
    bool skip_ok(uint64_t g) const;
    void read_more();
    void demand_past_end();
    void settle();  // a whole-file inflate started by the constructor: wait for it, or fall back
    struct Whole {
        bool ok = false;
        char* p = nullptr;
        size_t n = 0, cap = 0;
    };
    std::future<Whole> whole_;  // (.gz, not BGZF: libdeflate inflating the whole file on a thread)
    std::string path_;
    gzFile gz_ = nullptr;
    std::unique_ptr<BgzfSource> bgzf_;  // BGZF input: members inflated on several threads
    std::unique_ptr<ParGzSource> pargz_;  // single-stream gzip: chunks inflated on several threads
    std::unique_ptr<GzAhead> gz_ahead_;  // other gzip: inflated on a thread of its own, ahead of the parser
    FILE* fp_ = nullptr;
    bool phred64_;
    uint64_t bsize_;
    bool eof_ = false;
    bool src_failed_ = false, src_reported_ = false;  // the gzip source failed / the parser got there
    int64_t src_hit_ = -1;
    size_t calls_ = 0;    // records read since begin() (read() calls, read_fast records)
    uint64_t total_ = 0;  // stream bytes read so far (the stream's size once eof_)
    ByteBuf* text_ = nullptr;
    uint64_t base_ = 0;   // stream offset of (*text_)[0]
    size_t pos_ = 0;      // arena offset of the next unread line
    std::string carry_;
    uint64_t carry_off_ = 0;
    std::vector<uint64_t> tidx_;  // bit i of word w: arena byte 64 (tbase_ + w) + i is '\r' or '\n'
    size_t tbase_ = 0, indexed_ = 0;
    char* map_ = nullptr;  // a regular file is read through a private mapping (zero copy)
    size_t map_size_ = 0;
    size_t map_cap_ = 0;   // (an inflated .gz: the anonymous mapping's reserved size)
    size_t avg_rec_ = 0;   // mean record bytes seen by read_fast (sizes its next region)
    std::string err_;
};

// Minimal fork-join pool: run(n, fn) calls fn(0..n-1) on the workers and the calling thread and
// returns when all are done.  Several threads may call run concurrently.
class Pool {
   public:
    explicit Pool(int workers);
    ~Pool();
    Pool(const Pool&) = delete;
    Pool& operator=(const Pool&) = delete;
    void run(int n, const std::function<void(int)>& fn);
    int size() const { return workers_ + 1; }

   private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
    int workers_;
};

// One pack of reads (pairs when paired): record text + the engine's batch planes + the engine's
// per-read records.  A pinned pack keeps planes, lengths and records in page-locked memory.
struct Pack {
    explicit Pack(bool pinned = false)
        : seq{ByteBuf(pinned), ByteBuf(pinned)},
          qual{ByteBuf(pinned), ByteBuf(pinned)},
          len{PodBuf<uint16_t>(pinned), PodBuf<uint16_t>(pinned)},
          flags(pinned),
          res(pinned),
          trec{PodBuf<fq_text_rec>(pinned), PodBuf<fq_text_rec>(pinned)},
          out_text{ByteBuf(pinned), ByteBuf(pinned)} {}
    int n = 0;
    int stride = 0;
    bool paired = false;
    ByteBuf text[2];           // arenas of buffered (gzip / pipe) input
    const char* base[2] = {nullptr, nullptr};  // what each mate's record offsets refer to
    std::vector<Rec> rec[2];
    ByteBuf seq[2], qual[2];  // batch planes
    PodBuf<uint16_t> len[2];
    PodBuf<uint8_t> flags;       // per-pair FQ_BF_* flags (index filter), sent when use_flags
    bool use_flags = false;
    PodBuf<fq_read_result> res;  // engine records: n (SE) or 2n (PE)
    uint64_t seq_no = 0;
    int max_cycles = 0;  // the engine parameters' max_cycles this pack was submitted with

    // FASTQ-text pack (fq_engine_submit_text, pack_text): each mate's text span (inside its arena or
    // the file mapping), the per-record index into it, and the output text the engine writes back
    bool text_mode = false;
    const char* span[2] = {nullptr, nullptr};
    uint64_t span_bytes[2] = {0, 0};
    PodBuf<fq_text_rec> trec[2];
    ByteBuf out_text[2];
    fq_text_out tout{};
    int max_len[2] = {0, 0};

    // raw-stream pack (fq_engine_raw_*): the engine cut the records from the input bytes; its
    // trimmed-adapter entries follow the output text in out_text[m]; its staging window is recycled
    // once the pack is reported
    bool raw = false;
    fq_raw_out rout{};
    int stage = -1;  // the raw driver's staging window of the pack's input bytes
    // records-only egress (fq_raw_out.results): the records and line offsets came back, the host
    // formats from its staging window (rbuf[m]: [carry capacity - rcin | window bytes rwin] in the
    // device buffer's layout; the carry is copied in front by the formatter from the previous pack)
    bool recs = false;
    char* rbuf[2] = {nullptr, nullptr};
    uint64_t rwin[2] = {0, 0}, rcin[2] = {0, 0}, rccap = 0;
    std::function<void(int)> stage_release;  // (records-only: the formatter returns stages through it)
    // records-only egress to plain outputs (zero copy): each mate's output is a list of byte ranges
    // -- runs of records that pass untrimmed, straight from the staging window, and the trimmed
    // records formatted into out_text[m] -- written with writev; `hold` keeps the window until the
    // writers are through with it
    bool zc = false;
    std::vector<iovec> segs[2];
    std::shared_ptr<void> hold;

    // -c: pairs whose bases the engine corrected read their seq/qual from a corrected copy
    // (fix[i] -> seq1 qual1 seq2 qual2 back to back; nullptr = the original text)
    std::vector<const char*> fix;
    std::vector<std::string> fix_arena;

    const char* arena(int m) const { return base[m]; }
    const char* name(int m, size_t i) const { return arena(m) + rec[m][i].off; }
    const char* seq_text(int m, size_t i) const {
        if (!fix.empty() && fix[i]) return fix[i] + (m ? 2 * (size_t)rec[0][i].len : 0);
        return arena(m) + rec[m][i].seq_off();
    }
    const char* strand(int m, size_t i) const { return arena(m) + rec[m][i].strand_off(); }
    const char* qual_text(int m, size_t i) const {
        if (!fix.empty() && fix[i]) return fix[i] + (m ? 2 * (size_t)rec[0][i].len + rec[1][i].len : rec[0][i].len);
        return arena(m) + rec[m][i].qual_off();
    }
    void clear();
    fq_batch batch() const;
    fq_read_result* results() {  // sized for this pack
        res.resize((size_t)n * (paired ? 2 : 1));
        return res.data();
    }
};

// Fills the pack's lengths, stride and tile planes from its record text (pool-parallel over
// whole tiles when a pool is given).  Throws on reads longer than 65535 bases.
void pack_tiles(Pack& pk, Pool* pool);

// The FASTQ-text form of a pack (fq_engine_submit_text): each mate's span of text, one
// fq_text_rec per record, the planes' stride and the output buffers; no planes are built on the
// host.  False (the pack then goes through pack_tiles) when a span exceeds 4 GiB or a line 65535
// bytes.
// merged: -m (PE), whose output is the merged stream in out_text[0] (both mates' text plus a
// merged name's tag per pair; out_text[1] only takes the engine's adapter entries).
bool pack_text(Pack& pk, Pool* pool, bool merged = false);

// Reads up to max_n records (pairs) into a pack and builds its planes.  Two-file PE input is
// parsed by two threads, one per mate, with the reference's stop rule and messages (the pair
// reader stops at the first mate that fails, src/fqreader.cpp:254-267).
// Returns false when no record could be read.
class PackReader {
   public:
    PackReader(const std::string& in1, const std::string& in2, bool interleaved, bool phred64,
               int buf_size = 1 << 20);
    bool next(Pack& pk, size_t max_n, Pool* pool = nullptr);
    bool paired() const { return paired_; }
    uint64_t reads_seen() const { return reads_; }
    // continue at stream offsets off1 / off2 (where the GPU's raw stream stopped: mapped regular
    // files, or single-stream gzip files not read yet), numbering packs from first_seq
    void seek(uint64_t off1, uint64_t off2, uint64_t first_seq);
    bool mapped() { return r1_.mapped() && (!r2_ || r2_->mapped()); }
    bool parallel_gz() const { return r1_.parallel_gz() && (!r2_ || r2_->parallel_gz()); }
    double parse_s = 0, tiles_s = 0;  // time spent parsing records / filling batch planes
    bool defer_tiles = false;         // next() leaves pack_tiles to the caller (another thread)

   private:
    FqBulkReader r1_;
    std::unique_ptr<FqBulkReader> r2_;
    bool paired_, interleaved_;
    bool done_ = false;
    uint64_t reads_ = 0, packs_ = 0;
};

// An output file.  Plain files take the text as is.  Gzip output (src/writer.cpp:36-47, level
// -z) is one gzip member per block of text, the blocks compressed independently (in parallel
// on a pool when one is given): a valid multi-member gzip file whose decompressed bytes are the
// reference's.
class Writer {
   public:
    Writer(const std::string& path, int level);
    ~Writer();
    Writer(const Writer&) = delete;
    Writer& operator=(const Writer&) = delete;
    void write(const std::vector<std::string>& blocks, Pool* pool = nullptr);
    void write(const std::string& s) { write(std::vector<std::string>{s}); }
    // n bytes from p as they are (gzip: in blocks compressed in parallel on the pool)
    void write_raw(const char* p, size_t n, Pool* pool = nullptr);
    // plain outputs only: the byte ranges in order (writev)
    void write_segs(const iovec* v, size_t n);
    bool gzip() const { return gzip_; }
    // Plain regular files are written with pwrite at offsets claimed in output order (no stdio
    // buffer), so several threads can write claimed ranges at once (AsyncWriter); claim() is
    // called in order by one thread, write_at / write_segs_at from any.
    bool positional() const { return positional_; }
    uint64_t claim(size_t n) {
        const uint64_t o = off_;
        off_ += n;
        return o;
    }
    void write_at(uint64_t off, const char* p, size_t n);
    void write_segs_at(uint64_t off, const iovec* v, size_t n);
    void close();  // flushes; throws on a short write or a failed close (full disk)

   private:
    FILE* fp_ = nullptr;
    bool gzip_ = false;
    bool positional_ = false;
    uint64_t off_ = 0;
    bool any_member_ = false;
    int level_ = 4;
};

}  // namespace fqhost
