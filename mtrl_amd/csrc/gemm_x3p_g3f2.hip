// gemm_x3p_g3f2.hip -- instantiation unit of the plane GEMM: GeoBig16, operand-form mask 4
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g3f2, GeoBig16, 4)
}  // namespace mtsac
