// Internal view of the RCCL communicator (public API in include/mmad.h).
#pragma once
#include "../../include/mmad.h"

int mmad_comm_size(const mmad_comm* c);
// two in-place fp32 sum all-reduces issued as ONE RCCL group (one launch,
// one collective latency): the DP step's small bucket and its loss scalar
int mmad_allreduce_pair(mmad_comm* c, float* a, int64_t na, float* b, int64_t nb, void* stream);
