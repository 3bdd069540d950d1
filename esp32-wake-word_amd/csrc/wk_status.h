// wk_status.h -- error reporting shared by the C-ABI translation units of both
// libraries (internal).  libwakeword.so defines these in wk_api.hip,
// libwakeword_host.so in wk_host.cpp; plain C++, no HIP.
#pragma once
#include <string>

#include "wakeword.h"

namespace wk {

extern thread_local std::string g_last_error;   // read back by wk_last_error() / wkh_last_error()
wk_status invalid(const char* what);
wk_status fail(wk_status s, const char* what);

}  // namespace wk
