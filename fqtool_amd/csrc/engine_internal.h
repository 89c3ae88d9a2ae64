// engine_internal.h -- launch entry points shared between the engine's translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/fqengine.h"

size_t fq_pack_kernel_lds_bytes(const fq_params& p);
hipError_t fq_pack_kernel_set_lds(const fq_params& p);
hipError_t fq_launch_pack_kernel(const fq_params& p, const fq_batch& b, fq_read_result* res, unsigned long long* acc,
                                 int* err, int grid, hipStream_t stream);
hipError_t fq_launch_synth(const fq_batch& b, uint64_t seed, uint64_t first_index, int read_len, hipStream_t stream);
