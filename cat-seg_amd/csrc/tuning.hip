// Registry behind include/catseg_hip_tuning.h: each kernel file registers its A/B knobs
// (process-wide ints read at launch) with CATSEG_KNOB; one C entry sets / reads them by name.
#include <string.h>
#include <string>
#include "catseg_hip_tuning.h"
#include "capi.h"

namespace {
struct Knob { const char* name; int* value; };
constexpr int kMaxKnobs = 64;
Knob* table() { static Knob t[kMaxKnobs]; return t; }
int& count() { static int n = 0; return n; }
int* find(const char* name) {
  if (!name) return nullptr;
  for (int i = 0; i < count(); ++i)
    if (strcmp(table()[i].name, name) == 0) return table()[i].value;
  return nullptr;
}
}  // namespace

CatsegKnobReg::CatsegKnobReg(const char* name, int* value) {
  if (count() < kMaxKnobs) table()[count()++] = Knob{name, value};
}

extern "C" int catseg_tuning_set(const char* name, int value) {
  int* p = find(name);
  if (!p) {
    catseg_set_error("tuning: unknown knob '%s'", name ? name : "(null)");
    return CATSEG_ERR_ARG;
  }
  *p = value;
  return CATSEG_OK;
}

extern "C" int catseg_tuning_get(const char* name, int* value) {
  int* p = find(name);
  if (!p || !value) {
    catseg_set_error("tuning: unknown knob '%s'", name ? name : "(null)");
    return CATSEG_ERR_ARG;
  }
  *value = *p;
  return CATSEG_OK;
}

extern "C" const char* catseg_tuning_list(void) {
  static std::string s;
  s.clear();
  for (int i = 0; i < count(); ++i) {
    if (i) s += ",";
    s += table()[i].name;
  }
  return s.c_str();
}
