// time.Time.Format(time.RFC3339Nano) of a UTC instant (Now() in the Stage templates), shared by
// the host renderer (patch.cpp) and the device emitter (emit.hip)
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>

namespace kwkfmt {

inline std::string rfc3339nano(int64_t ns) {
  int64_t sec = ns / 1000000000, frac = ns % 1000000000;
  if (frac < 0) { frac += 1000000000; sec -= 1; }
  int64_t days = sec / 86400, rem = sec % 86400;
  if (rem < 0) { rem += 86400; days -= 1; }
  // civil_from_days (proleptic Gregorian)
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const int64_t doe = days - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t d = doy - (153 * mp + 2) / 5 + 1;
  const int64_t m = mp < 10 ? mp + 3 : mp - 9;
  if (m <= 2) ++y;
  char buf[64];
  snprintf(buf, sizeof buf, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)m, (long long)d,
           (long long)(rem / 3600), (long long)(rem / 60 % 60), (long long)(rem % 60));
  std::string s(buf);
  if (frac) {
    snprintf(buf, sizeof buf, ".%09lld", (long long)frac);
    std::string f(buf);
    while (f.back() == '0') f.pop_back();
    s += f;
  }
  return s + "Z";
}

}  // namespace kwkfmt
