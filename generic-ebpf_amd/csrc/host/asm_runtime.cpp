// asm_runtime.cpp — loader for the hand-written gfx950 assembly interpreter (variant 0).
// Placeholder until the assembly kernel lands: reports it unavailable so launches use the
// portable HIP interpreter (variant 1).
#include <hip/hip_runtime.h>

#include "internal.h"

int
asm_available(int)
{
	return 0;
}

int
asm_link_entries(int, std::vector<dp_entry> &)
{
	return ENOSYS;
}

hipError_t
launch_interp_asm(const dp_launch &, hipStream_t, int)
{
	return hipErrorNotSupported;
}
