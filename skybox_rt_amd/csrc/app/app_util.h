// app_util.h -- helpers shared by the host apps in librtapp.so (rt_app.cpp
// owns the thread's last-error string behind rt_last_error()).
#pragma once

#include <string>

namespace rtapp {
int set_error(const std::string& message, int code = -1);  // returns code
std::string library_dir();                                 // directory of librtapp.so
}  // namespace rtapp
