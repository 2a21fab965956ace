// gemm_x3p_g5in.hip -- instantiation unit of the plane GEMM: GeoTall224In (input-layer forward, mask 4)
#include "gemm_x3p_impl.h"

namespace mtsac {
X3P_UNIT(x3p_unit_g5in, GeoTall224In, 4)
}  // namespace mtsac
