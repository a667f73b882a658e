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

// resource.Format: how a quantity prints (apimachinery quantity.go).  Parse takes it from the
// suffix: Ki..Ei -> BinarySI, e<N>/E<N> exponent -> DecimalExponent, none or n..E -> DecimalSI.
enum class Format { kDecimalExponent, kBinarySI, kDecimalSI };

class Quantity {
 public:
  Quantity() = default;
  static Quantity Parse(const std::string& s);     // throws QuantityError
  static Quantity MustParse(const std::string& s) { return Parse(s); }
  // From an engine result.  Default format: DecimalSI for cpu, BinarySI for everything else.
  static Quantity FromCanonical(const std::string& resource, int64_t v);
  static Quantity FromCanonical(const std::string& resource, int64_t v, Format f);

  // canonical int64 for `resource` (cpu: milli); throws QuantityError when inexact / negative / > int64
  int64_t Canonical(const std::string& resource) const;
  // Key tables (placement.h pe_pg_min_resources_keys): the value as an exact count of 10^s units.
  // Exp10(): the exponent e of value = m * 10^e, m an integer not divisible by 10 (0 for zero) -- the
  // finest scale the value needs.  Scaled(s): value / 10^s when that is an exact int64 in [0, INT64_MAX]
  // (s <= Exp10()), else nullopt (negative, or no int64: Go would hold the sum in inf.Dec).
  int Exp10() const;
  std::optional<int64_t> Scaled(int s) const;
  static Quantity FromScaled(int64_t v, int s, Format f);
  Quantity WithFormat(Format f) const {
    Quantity q = *this;
    q.format_ = f;
    return q;
  }
  bool Negative() const { return mant_ < 0; }
  // Cmp == 0 semantics
  bool Equal(const Quantity& o) const;
  bool IsZero() const { return mant_ == 0; }
  Format format() const { return format_; }
  // Go's Quantity.String(): CanonicalizeBytes of the value in its format (quantity.go) --
  // BinarySI prints as <n>Ki..Ei when |v| >= 1024 and v is an integer, else falls back to
  // DecimalSI; DecimalSI / DecimalExponent strip factors of ten and round the exponent down to a
  // multiple of 3 (n u m "" k M G T P E, or e<N>).  "1.5Gi" -> "1536Mi", "1000m" -> "1",
  // "0.5" -> "500m", "1024Mi" -> "1Gi", "1e3" -> "1e3".  What the JSON encoder writes.
  std::string String() const;

 private:
  // value = mant * 10^e10 * 2^e2, mant signed
  __int128 mant_ = 0;
  int e10_ = 0;
  int e2_ = 0;
  Format format_ = Format::kDecimalSI;
};

using ResourceList = std::map<std::string, Quantity>;

bool EqualResourceList(const ResourceList& a, const ResourceList& b);

}  // namespace kf
