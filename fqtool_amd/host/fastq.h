// fastq.h -- FASTQ input and output of the host tool.
//
// FqReader restates the reference reader (src/fqreader.cpp:3-195): 1 MiB buffered lines over
// zlib or stdio, a line ends at '\r' or '\n' ("\r\n" counts once), records start at the next
// line beginning with '@', phred64 qualities are shifted at parse time (src/read.h:71-75) and a
// quality/sequence length mismatch silently ends the input (src/fqreader.cpp:184-191).
// Records are appended to a Pack: the engine's SoA rows (fq_batch) plus the name/strand text
// the writer needs.  Writer restates src/writer.cpp (gzip level -z with a 1 MiB gzbuffer, or a
// plain file).
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fqengine.h"

namespace fqhost {

class FqReader {
   public:
    FqReader(const std::string& path, bool phred64);
    ~FqReader();
    FqReader(const FqReader&) = delete;
    FqReader& operator=(const FqReader&) = delete;
    // Next record; false at end of input (or on a quality/sequence length mismatch).
    bool read(std::string& name, std::string& seq, std::string& strand, std::string& qual);

   private:
    bool get_line(std::string& out);
    void fill();
    bool at_eof() const;
    gzFile gz_ = nullptr;
    FILE* fp_ = nullptr;
    bool phred64_;
    std::vector<char> buf_;
    int len_ = 0, used_ = 0;
    bool eof_ = false;
};

// One pack of reads (pairs when paired): the engine's batch planes (chunk-interleaved tiles,
// include/fqengine.h) + the records' text fields, kept for output formatting.
struct Pack {
    int n = 0;
    int stride = 0;
    bool paired = false;
    std::vector<uint8_t> seq[2], qual[2];  // batch planes
    std::vector<std::string> seq_text[2], qual_text[2];
    std::vector<uint16_t> len[2];
    std::vector<std::string> name[2], strand[2];
    uint64_t seq_no = 0;
    fq_batch batch() const;
};

// Reads up to max_n records (pairs) into a pack; rows are padded to a multiple of 16 bytes and
// the planes to whole tiles.
// Returns false when no record could be read.
class PackReader {
   public:
    PackReader(const std::string& in1, const std::string& in2, bool interleaved, bool phred64);
    bool next(Pack& pk, size_t max_n);
    bool paired() const { return paired_; }
    uint64_t reads_seen() const { return reads_; }

   private:
    FqReader r1_;
    FqReader* r2_ = nullptr;
    std::unique_ptr<FqReader> r2_own_;
    bool paired_, interleaved_;
    bool done_ = false;
    uint64_t reads_ = 0, packs_ = 0;
};

class Writer {
   public:
    Writer(const std::string& path, int level);
    ~Writer();
    void write(const std::string& s);

   private:
    gzFile gz_ = nullptr;
    FILE* fp_ = nullptr;
};

}  // namespace fqhost
