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
  q.text_ = s0;
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
  Quantity q;
  q.mant_ = v;
  q.e10_ = resource == "cpu" ? -3 : 0;
  if (resource == "cpu") {
    q.text_ = (v % 1000 == 0) ? std::to_string(v / 1000) : std::to_string(v) + "m";
  } else {
    static const char* suf[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
    int k = 0;
    int64_t m = v;
    while (m != 0 && k < 6 && m % 1024 == 0) {
      m /= 1024;
      ++k;
    }
    q.text_ = std::to_string(m) + suf[k];
  }
  return q;
}

bool Quantity::Equal(const Quantity& o) const {
  __int128 m1, m2;
  int a1, b1, a2, b2;
  normalize(mant_, e10_, e2_, &m1, &a1, &b1);
  normalize(o.mant_, o.e10_, o.e2_, &m2, &a2, &b2);
  return m1 == m2 && a1 == a2 && b1 == b2;
}

std::string Quantity::String() const {
  if (!text_.empty()) return text_;
  return "0";
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
