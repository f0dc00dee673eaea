// The reference's namespace on this library.  Every forwarding header under include/mscclpp includes
// this after its mscclpp_amd twin, so mscclpp::MemoryChannelDeviceHandle, mscclpp::LL16Packet,
// mscclpp::PortChannelDeviceHandle, mscclpp::collective::AlgorithmCollectionBuilder, ... name the
// mscclpp_amd declarations: a using-directive, not an alias, so one translation unit may include any
// mix of forwarding headers (an alias can be declared only once) and `using namespace mscclpp;`
// brings in the same names.  Declaring new members of namespace mscclpp (or specialising one of
// its templates under that spelling) is the one thing a caller must spell as mscclpp_amd.
#ifndef MSCCLPP_AMD_FWD_NAMESPACE_HPP_
#define MSCCLPP_AMD_FWD_NAMESPACE_HPP_

namespace mscclpp_amd {}
namespace mscclpp {
using namespace ::mscclpp_amd;
}  // namespace mscclpp

#endif  // MSCCLPP_AMD_FWD_NAMESPACE_HPP_
