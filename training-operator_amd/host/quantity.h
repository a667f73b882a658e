// k8s resource.Quantity, restricted to what the engine needs: exact parsing of the string forms
// (apimachinery v0.30.7 grammar: <signedNumber><suffix>, suffix binarySI | decimalSI | decimalExponent)
// and conversion to the canonical int64 unit of an engine dimension (cpu -> milli-cores,
// everything else -> base units).  Values that are not exactly representable are refused, as
// SURVEY.md Appendix A requires; equality is value equality (Quantity.Cmp == 0).
#pragma once
#include <stdint.h>

#include <map>
#include <optional>
#include <string>

namespace kf {

struct QuantityError {
  std::string msg;
};

class Quantity {
 public:
  Quantity() = default;
  static Quantity Parse(const std::string& s);     // throws QuantityError
  static Quantity MustParse(const std::string& s) { return Parse(s); }
  static Quantity FromCanonical(const std::string& resource, int64_t v);

  // canonical int64 for `resource` (cpu: milli); throws QuantityError when inexact / negative / > int64
  int64_t Canonical(const std::string& resource) const;
  // Cmp == 0 semantics
  bool Equal(const Quantity& o) const;
  std::string String() const;                         // an exact string form (not Go's canonical format)

 private:
  // value = mant * 10^e10 * 2^e2, mant signed
  __int128 mant_ = 0;
  int e10_ = 0;
  int e2_ = 0;
  std::string text_;
};

using ResourceList = std::map<std::string, Quantity>;

bool EqualResourceList(const ResourceList& a, const ResourceList& b);

}  // namespace kf
