// gemm_x3p_g1.hip -- instantiation unit of the plane GEMM: GeoWide, operand-form mask 15
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g1, GeoWide, 15)
}  // namespace mtsac
