// Internal view of the RCCL communicator (public API in include/mmad.h).
#pragma once
#include "../../include/mmad.h"

int mmad_comm_size(const mmad_comm* c);
