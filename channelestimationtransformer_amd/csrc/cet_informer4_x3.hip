// v4 fused Informer instances for the P_X3 operand policy (cet_informer4.hpp; one precision per
// translation unit so the instances compile in parallel).
#include "cet_informer4.hpp"

extern "C" int cet_launch_informer_v4_p1(const cet::InformerArgs* a, int dff, int lds_bytes, hipStream_t stream) {
  return cet::v4::launch_v4<cet::v4::P_X3>(a, dff, lds_bytes, stream);
}

#ifdef CET_AB8_DUMP
// diagnostic: read / clear the round-5 ab8 dump (cet_v4.hpp g_ab8_dump)
extern "C" int cet_ab8_dump(unsigned int* host, int clear) {
  if (clear) {
    static unsigned int z[8 * 128 * 64] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(cet::v4::g_ab8_dump), z, sizeof z) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(cet::v4::g_ab8_dump), 8 * 128 * 64 * 4) == hipSuccess ? 0 : -1;
}
#endif
