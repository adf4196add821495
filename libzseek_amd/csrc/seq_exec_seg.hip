// seq_exec_seg.hip — the execute kernel's block-route instantiation
// (seq_exec.hip, SEG = true: items read job by job) in a translation unit of
// its own, so the production instantiation's code is what it is alone.
#define ZSK_EXEC_SEG_TU 1
#include "seq_exec.hip"
