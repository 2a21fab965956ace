// gemm_x3p_g4.hip -- instantiation unit of the plane GEMM: GeoSmall16, operand-form mask 15
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g4, GeoSmall16, 15)
}  // namespace mtsac
