// gemm_x3p_g3f3.hip -- instantiation unit of the plane GEMM: GeoBig16, operand-form mask 8
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g3f3, GeoBig16, 8)
}  // namespace mtsac
