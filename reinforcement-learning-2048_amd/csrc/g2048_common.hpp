// g2048_common.hpp -- internal helpers shared by the translation units of libg2048.so.
#pragma once

// Record a printf-style message for g2048_last_error() and return `code` (hidden symbol).
int g2048_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
