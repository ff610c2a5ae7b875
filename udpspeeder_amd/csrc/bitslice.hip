// bitslice.hip -- placeholder until the generated bit-sliced kernels land.
#include "rsmi_internal.hpp"
namespace rsmi {
bool has_bitslice(int, int) { return false; }
hipError_t launch_encode_bitslice(const UniformArgs &, hipStream_t) { return hipErrorNotSupported; }
}  // namespace rsmi
