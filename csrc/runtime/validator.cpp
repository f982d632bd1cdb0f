#include "validator.h"

#include <charconv>
#include <cmath>
#include <cstring>

namespace xgs {

std::string rust_f32_display(float v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char buf[128];
  // Shortest representation that round-trips, in fixed notation == Rust's
  // `impl Display for f32` (which never switches to exponent form).
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::fixed);
  std::string s(buf, r.ptr);
  if (s == "-0") return "-0";
  return s;
}

// Decode one code point; returns bytes consumed (>=1). Invalid sequences are
// consumed one byte at a time and treated as non-whitespace.
static size_t decode_utf8(const unsigned char* p, size_t n, uint32_t& cp) {
  unsigned char c = p[0];
  if (c < 0x80) { cp = c; return 1; }
  size_t len = (c >> 5) == 0x6 ? 2 : (c >> 4) == 0xE ? 3 : (c >> 3) == 0x1E ? 4 : 0;
  if (len == 0 || len > n) { cp = 0xFFFD; return 1; }
  cp = c & (0xFF >> (len + 1));
  for (size_t i = 1; i < len; ++i) {
    if ((p[i] & 0xC0) != 0x80) { cp = 0xFFFD; return 1; }
    cp = (cp << 6) | (p[i] & 0x3F);
  }
  return len;
}

// Unicode White_Space property (what Rust's char::is_whitespace tests).
static bool is_unicode_ws(uint32_t c) {
  if (c >= 0x09 && c <= 0x0D) return true;
  switch (c) {
    case 0x20: case 0x85: case 0xA0: case 0x1680: case 0x2028: case 0x2029:
    case 0x202F: case 0x205F: case 0x3000:
      return true;
    default:
      return c >= 0x2000 && c <= 0x200A;
  }
}

bool is_blank_utf8(const std::string& s) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  size_t n = s.size(), i = 0;
  while (i < n) {
    uint32_t cp;
    size_t k = decode_utf8(p + i, n - i, cp);
    if (!is_unicode_ws(cp)) return false;
    i += k;
  }
  return true;
}

static ValidationResult empty_prompt() {
  ValidationResult r;
  r.kind = ValidationKind::EmptyPrompt;
  r.message = "Empty prompt not allowed";
  return r;
}

static ValidationResult missing(const std::string& f) {
  ValidationResult r;
  r.kind = ValidationKind::MissingField;
  r.field = f;
  r.message = "Missing required field: " + f;
  return r;
}

static ValidationResult token_limit(size_t actual, size_t limit) {
  ValidationResult r;
  r.kind = ValidationKind::TokenLimitExceeded;
  r.actual = actual;
  r.limit = limit;
  r.message = "Token limit exceeded: " + std::to_string(actual) + " tokens > " +
              std::to_string(limit) + " max";
  return r;
}

static ValidationResult invalid_param(const std::string& f, const std::string& reason) {
  ValidationResult r;
  r.kind = ValidationKind::InvalidParameter;
  r.field = f;
  r.reason = reason;
  r.message = "Invalid parameter '" + f + "': " + reason;
  return r;
}

ValidationResult RequestValidator::check_sampling(size_t max_tokens, float temperature,
                                                  float top_p) const {
  if (max_tokens > cfg_.max_output_tokens)
    return invalid_param("max_tokens", "must be <= " + std::to_string(cfg_.max_output_tokens) +
                                           ", got " + std::to_string(max_tokens));
  bool t_bad = temperature < cfg_.min_temperature || temperature > cfg_.max_temperature ||
               (cfg_.reject_nan && std::isnan(temperature));
  if (t_bad)
    return invalid_param("temperature", "must be between " + rust_f32_display(cfg_.min_temperature) +
                                            " and " + rust_f32_display(cfg_.max_temperature) +
                                            ", got " + rust_f32_display(temperature));
  bool p_bad = top_p < cfg_.min_top_p || top_p > cfg_.max_top_p ||
               (cfg_.reject_nan && std::isnan(top_p));
  if (p_bad)
    return invalid_param("top_p", "must be between " + rust_f32_display(cfg_.min_top_p) + " and " +
                                      rust_f32_display(cfg_.max_top_p) + ", got " +
                                      rust_f32_display(top_p));
  return ValidationResult{};
}

ValidationResult RequestValidator::validate_generate(const std::string& prompt, size_t max_tokens,
                                                     float temperature, float top_p) const {
  if (is_blank_utf8(prompt)) return empty_prompt();
  size_t n = token_count(prompt);
  if (n > cfg_.max_context_tokens) return token_limit(n, cfg_.max_context_tokens);
  return check_sampling(max_tokens, temperature, top_p);
}

ValidationResult RequestValidator::validate_chat(const std::vector<std::string>& contents,
                                                 size_t max_tokens, float temperature,
                                                 float top_p) const {
  if (contents.empty()) return missing("messages");
  bool has = false;
  for (const auto& c : contents)
    if (!is_blank_utf8(c)) { has = true; break; }
  if (!has) return empty_prompt();
  size_t total = 0;
  for (const auto& c : contents) total += token_count(c);
  if (total > cfg_.max_context_tokens) return token_limit(total, cfg_.max_context_tokens);
  return check_sampling(max_tokens, temperature, top_p);
}

ValidationResult RequestValidator::validate_embeddings(const std::vector<std::string>& inputs) const {
  if (inputs.empty()) return missing("input");
  for (size_t i = 0; i < inputs.size(); ++i) {
    if (is_blank_utf8(inputs[i]))
      return invalid_param("input[" + std::to_string(i) + "]", "cannot be empty");
    size_t n = token_count(inputs[i]);
    if (n > cfg_.max_context_tokens) return token_limit(n, cfg_.max_context_tokens);
  }
  return ValidationResult{};
}

}  // namespace xgs
