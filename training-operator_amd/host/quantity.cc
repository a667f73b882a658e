#include "quantity.h"

#include <cctype>

namespace kf {

namespace {

constexpr __int128 kI128Max = (((__int128)1) << 125);

int suffix_exp(const std::string& suf, int* e10, int* e2) {
  static const std::map<std::string, int> bin = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  static const std::map<std::string, int> dec = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                 {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  *e10 = 0;
  *e2 = 0;
  auto b = bin.find(suf);
  if (b != bin.end()) {
    *e2 = b->second;
    return 0;
  }
  auto d = dec.find(suf);
  if (d != dec.end()) {
    *e10 = d->second;
    return 0;
  }
  if (suf.size() >= 2 && (suf[0] == 'e' || suf[0] == 'E')) {
    size_t i = 1;
    bool neg = false;
    if (suf[i] == '+' || suf[i] == '-') neg = suf[i++] == '-';
    if (i >= suf.size()) return -1;
    int v = 0;
    for (; i < suf.size(); ++i) {
      if (!isdigit((unsigned char)suf[i]) || v > 10000) return -1;
      v = v * 10 + (suf[i] - '0');
    }
    *e10 = neg ? -v : v;
    return 0;
  }
  return -1;
}

void normalize(__int128 mant, int e10, int e2, __int128* m, int* a2, int* a5) {
  // value = mant * 2^(e2 + e10) * 5^e10, strip the 2s and 5s out of mant
  *a2 = e2 + e10;
  *a5 = e10;
  if (mant == 0) {
    *m = 0;
    *a2 = *a5 = 0;
    return;
  }
  while (mant % 2 == 0) {
    mant /= 2;
    ++*a2;
  }
  while (mant % 5 == 0) {
    mant /= 5;
    ++*a5;
  }
  *m = mant;
}

}  // namespace

Quantity Quantity::Parse(const std::string& s0) {
  std::string s;
  for (char c : s0)
    if (!isspace((unsigned char)c)) s.push_back(c);
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  __int128 mant = 0;
  int digits = 0, frac = 0;
  bool seen_dot = false;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (isdigit((unsigned char)c)) {
      if (mant > kI128Max / 10) throw QuantityError{"quantity too large: " + s0};
      mant = mant * 10 + (c - '0');
      ++digits;
      if (seen_dot) ++frac;
    } else if (c == '.' && !seen_dot) {
      seen_dot = true;
    } else {
      break;
    }
  }
  if (digits == 0) throw QuantityError{"quantities must match the regular expression: " + s0};
  int e10, e2;
  if (suffix_exp(s.substr(i), &e10, &e2) != 0) throw QuantityError{"unable to parse quantity's suffix: " + s0};
  Quantity q;
  q.mant_ = neg ? -mant : mant;
  q.e10_ = e10 - frac;
  q.e2_ = e2;
  const std::string suf = s.substr(i);
  q.format_ = e2 ? Format::kBinarySI
                 : (suf.size() >= 2 && (suf[0] == 'e' || suf[0] == 'E')) ? Format::kDecimalExponent : Format::kDecimalSI;
  return q;
}

int64_t Quantity::Canonical(const std::string& resource) const {
  __int128 x = mant_;
  if (x < 0) throw QuantityError{resource + "=" + String() + " is negative"};
  const int E = e10_ + (resource == "cpu" ? 3 : 0);
  for (int k = 0; k < e2_; ++k) {
    if (x > kI128Max / 2) throw QuantityError{resource + "=" + String() + " does not fit int64"};
    x *= 2;
  }
  for (int k = 0; k < E; ++k) {
    if (x > kI128Max / 10) throw QuantityError{resource + "=" + String() + " does not fit int64"};
    x *= 10;
  }
  for (int k = 0; k < -E; ++k) {
    if (x % 10 != 0) throw QuantityError{resource + "=" + String() + " is not an exact canonical integer"};
    x /= 10;
  }
  if (x > (__int128)INT64_MAX) throw QuantityError{resource + "=" + String() + " does not fit int64"};
  return (int64_t)x;
}

Quantity Quantity::FromCanonical(const std::string& resource, int64_t v) {
  return FromCanonical(resource, v, resource == "cpu" ? Format::kDecimalSI : Format::kBinarySI);
}

Quantity Quantity::FromCanonical(const std::string& resource, int64_t v, Format f) {
  Quantity q;
  q.mant_ = v;
  q.e10_ = resource == "cpu" ? -3 : 0;
  q.format_ = f;
  return q;
}

int Quantity::Exp10() const {
  if (mant_ == 0) return 0;
  // value = mant * 2^e2 * 10^e10 (e2 >= 0): trailing zeros of mant * 2^e2 = min(2s, 5s) of it
  __int128 m = mant_ < 0 ? -mant_ : mant_;
  int twos = e2_, fives = 0;
  while (m % 2 == 0) {
    m /= 2;
    ++twos;
  }
  while (m % 5 == 0) {
    m /= 5;
    ++fives;
  }
  return e10_ + (twos < fives ? twos : fives);
}

std::optional<int64_t> Quantity::Scaled(int s) const {
  if (mant_ < 0) return std::nullopt;
  if (mant_ == 0) return 0;
  if (s > Exp10()) return std::nullopt;   // (not an integer count of 10^s)
  __int128 x = mant_;
  int k = e10_ - s;                       // value / 10^s = mant * 2^e2 * 10^k
  while (k < 0 && x % 10 == 0) {          // the exact divisions first: x never grows past the result
    x /= 10;
    ++k;
  }
  for (int i = 0; i < e2_; ++i) {
    if (x > (__int128)INT64_MAX) return std::nullopt;
    x *= 2;
  }
  while (k < 0) {                         // (the 2s of 2^e2 pair with the 5s left in x)
    x /= 10;
    ++k;
  }
  for (; k > 0; --k) {
    if (x > (__int128)INT64_MAX) return std::nullopt;
    x *= 10;
  }
  if (x > (__int128)INT64_MAX) return std::nullopt;
  return (int64_t)x;
}

Quantity Quantity::FromScaled(int64_t v, int s, Format f) {
  Quantity q;
  q.mant_ = v;
  q.e10_ = s;
  q.format_ = f;
  return q;
}

bool Quantity::Equal(const Quantity& o) const {
  __int128 m1, m2;
  int a1, b1, a2, b2;
  normalize(mant_, e10_, e2_, &m1, &a1, &b1);
  normalize(o.mant_, o.e10_, o.e2_, &m2, &a2, &b2);
  return m1 == m2 && a1 == a2 && b1 == b2;
}

static std::string i128_str(__int128 x) {
  if (x == 0) return "0";
  const bool neg = x < 0;
  std::string s;
  for (; x != 0; x /= 10) s.push_back((char)('0' + (int)(neg ? -(x % 10) : x % 10)));
  if (neg) s.push_back('-');
  return std::string(s.rbegin(), s.rend());
}

std::string Quantity::String() const {
  // quantity.go CanonicalizeBytes (apimachinery v0.30.7), restated for the exact value
  // mant * 10^e10 * 2^e2 (e2 >= 0).
  if (mant_ == 0) return "0";
  __int128 a = mant_;                          // value = a * 10^x
  for (int k = 0; k < e2_; ++k) a *= 2;
  int x = e10_;
  Format f = format_;
  if (f == Format::kBinarySI) {
    // |v| < 1024 or not an integer: DecimalSI ("This avoids rounding" / "Don't lose precision")
    __int128 n = a;
    bool integer = true;
    for (int k = 0; k < x; ++k) n *= 10;
    for (int k = 0; k < -x && integer; ++k) {
      if (n % 10 != 0) integer = false;
      n /= 10;
    }
    if (!integer || (n > -1024 && n < 1024)) {
      f = Format::kDecimalSI;
    } else {
      static const char* bin[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
      int e = 0;                               // AsCanonicalBase1024Bytes: removeInt64Factors(v, 1024)
      __int128 m = n < 0 ? -n : n;
      while (m >= 1024 && m % 1024 == 0 && e < 6) {
        m /= 1024;
        ++e;
      }
      return i128_str(n < 0 ? -m : m) + bin[e];
    }
  }
  // AsCanonicalBytes: move factors of ten into the exponent, then make it a multiple of 3
  __int128 m = a < 0 ? -a : a;
  while (m >= 10 && m % 10 == 0) {
    m /= 10;
    ++x;
  }
  switch (x % 3) {                             // Go's % keeps the dividend's sign
    case 1: case -2: m *= 10; x -= 1; break;
    case 2: case -1: m *= 100; x -= 2; break;
    default: break;
  }
  const std::string num = i128_str(a < 0 ? -m : m);
  if (f == Format::kDecimalExponent) return x == 0 ? num : num + "e" + std::to_string(x);
  switch (x) {                                 // decimal SI suffixes (suffix.go)
    case -9: return num + "n";
    case -6: return num + "u";
    case -3: return num + "m";
    case 0: return num;
    case 3: return num + "k";
    case 6: return num + "M";
    case 9: return num + "G";
    case 12: return num + "T";
    case 15: return num + "P";
    case 18: return num + "E";
    default: return num + "e" + std::to_string(x);   // outside the SI table (no int64 canonical value)
  }
}

bool EqualResourceList(const ResourceList& a, const ResourceList& b) {
  if (a.size() != b.size()) return false;
  for (const auto& kv : a) {
    auto it = b.find(kv.first);
    if (it == b.end() || !kv.second.Equal(it->second)) return false;
  }
  return true;
}

}  // namespace kf
