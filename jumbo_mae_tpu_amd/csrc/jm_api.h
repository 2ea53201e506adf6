// Host-side argument structs shared by the kernel translation units and bindings.cpp.
#pragma once
#include <cstdint>

// Fused residual backward riding on the LayerNorm backward (layernorm.hip, LnResIO):
// for rows t >= T0, dy(b, t) = bf16(mask[b] * scale * dx(b, t)) at y/dy + b * yB + (t - T0) * yT,
// dscale += colsum(mask * dx * y), dbias += colsum(dy).  scale / mask / dscale / dbias may be null.
struct JmLnRes {
  const uint16_t* y;
  uint16_t* dy;
  long yB, yT;
  const float* scale;
  const float* mask;
  int T0;
  float* dscale;
  float* dbias;
};
