// evaluator.h -- host pre-pass: Evaluator::evaluateReadLen / evaluateAdapterSeq
// (reference src/evaluator.cpp:84-109, :229-446).
#pragma once

#include <string>

#include "../../include/fqhost.h"

namespace fqhost {

// longest of the first 1000 reads
int evaluate_read_len(const std::string& path);
// Evaluator::evaluateReadNum (src/evaluator.cpp:191-227): the record count when the file ends
// within 512 Ki records / 151 x 512 Ki bases, else an estimate from the bytes per record
int evaluate_read_num(const std::string& path);
// detected adapter of one mate file ("" when none), trim_tail1 = -t as the reference passes it.
// A read error message goes to *msgs when given (so two concurrent detections can report in
// the reference's order), else straight to stderr.
// The k-mer histogram and seed search run on HIP device `device` (fq_kmer_*), or on the backend
// given to set_kmer_backend.
std::string detect_adapter(const std::string& path, int trim_tail1, std::string* msgs = nullptr, int device = 0);
void set_kmer_backend(const struct fqh_kmer_backend* b);

}  // namespace fqhost
