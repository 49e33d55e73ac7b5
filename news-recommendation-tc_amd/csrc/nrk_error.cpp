// nrk_error.cpp -- thread-local last-error string of the C ABI.
#include <string>

#include "nrk_common.h"

namespace nrk {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }
}  // namespace nrk

extern "C" {
const char* nrk_last_error(void) { return nrk::g_last_error.c_str(); }
int nrk_abi_version(void) { return NRK_ABI_VERSION; }
}
