// NUMA placement with the reference's spellings (include/mscclpp/numa.hpp, src/core/numa.cc): the
// NUMA node of a GPU from its PCI device's sysfs entry (-1 if unknown), and pinning the calling
// thread to a node's CPUs (the proxy threads do this for their GPU, proxy.cc:23-33).  numaBind
// returns the node it bound to, or -1; the reference's returns nothing.
#pragma once

namespace mscclpp_amd {

int getDeviceNumaNode(int deviceId);
int numaBind(int node);

}  // namespace mscclpp_amd
