// pe_fast_long.hip -- the fast kernels of pe_fast.hip built again for reads of up to 320 bp
// (2x250 / 2x300 runs): 20 chunks per code column, one workgroup per CU (LDS), no merge variant
// (-m with rows longer than 160 bytes runs on the general kernel).  fq_launch_pe_fast picks this
// build for batches whose row stride exceeds 160.
#define FQ_MAXLEN 320
#define FQ_MAXLEN_BUILD_LONG 1
#include "pe_fast.hip"
