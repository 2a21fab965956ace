// gemm_x3p_g3f0.hip -- instantiation unit of the plane GEMM: GeoBig16, operand-form mask 1
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g3f0, GeoBig16, 1)
}  // namespace mtsac
