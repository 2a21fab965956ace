// gemm_x3p_g3in.hip -- instantiation unit of the plane GEMM: GeoBig16In, operand-form mask 15
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g3in, GeoBig16In, 15)
}  // namespace mtsac
