// gemm_x3p_g3f1.hip -- instantiation unit of the plane GEMM: GeoBig16, operand-form mask 2
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g3f1, GeoBig16, 2)
}  // namespace mtsac
