// Request admission validator.
//
// Behavioural parity with the reference `crates/core/src/validator.rs`:
//   * ValidatorConfig defaults (validator.rs:17-28): max_context_tokens=8192,
//     max_output_tokens=4096, temperature in [0,2], top_p in [0,1].
//   * token_count (validator.rs:60-65): 0 for "", else ceil(utf8_bytes / 4).
//   * validate_generate (validator.rs:68-122): first failing check wins, in the
//     order EmptyPrompt -> TokenLimitExceeded -> max_tokens -> temperature ->
//     top_p. "Empty" means Rust `str::trim()` leaves nothing, i.e. every code
//     point is Unicode White_Space.
//   * validate_chat (validator.rs:125-192): empty list -> MissingField
//     ("messages"); no non-blank content -> EmptyPrompt; sum of per-message
//     token_count -> TokenLimitExceeded; then the sampling checks.
//   * validate_embeddings (validator.rs:195-225): empty list ->
//     MissingField("input"); per item: blank -> InvalidParameter("input[i]",
//     "cannot be empty"), too long -> TokenLimitExceeded.
// Messages are formatted byte-identically to the Rust Display impls, including
// Rust's shortest-round-trip float formatting ("2", "2.5", "0.0000001").
// One deliberate difference: NaN temperature/top_p is rejected (the reference
// accepts it because both comparisons are false).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace xgs {

struct ValidatorConfig {
  size_t max_context_tokens = 8192;
  size_t max_output_tokens = 4096;
  float min_temperature = 0.0f;
  float max_temperature = 2.0f;
  float min_top_p = 0.0f;
  float max_top_p = 1.0f;
  bool reject_nan = true;
};

enum class ValidationKind : uint8_t {
  Ok = 0,
  InvalidJson = 1,
  MissingField = 2,
  TokenLimitExceeded = 3,
  InvalidParameter = 4,
  EmptyPrompt = 5,
};

struct ValidationResult {
  ValidationKind kind = ValidationKind::Ok;
  std::string field;    // MissingField / InvalidParameter
  std::string reason;   // InvalidParameter
  size_t actual = 0;    // TokenLimitExceeded
  size_t limit = 0;     // TokenLimitExceeded
  std::string message;  // full Display string
  bool ok() const { return kind == ValidationKind::Ok; }
};

// Rust `{}` Display of an f32 (shortest round-trip, fixed notation).
std::string rust_f32_display(float v);
// true iff every code point of the UTF-8 string is Unicode White_Space.
bool is_blank_utf8(const std::string& s);

class RequestValidator {
 public:
  explicit RequestValidator(ValidatorConfig cfg = ValidatorConfig()) : cfg_(cfg) {}

  size_t token_count(const std::string& text) const {
    return text.empty() ? 0 : (text.size() + 3) / 4;
  }

  ValidationResult validate_generate(const std::string& prompt, size_t max_tokens,
                                     float temperature, float top_p) const;
  ValidationResult validate_chat(const std::vector<std::string>& contents,
                                 size_t max_tokens, float temperature, float top_p) const;
  ValidationResult validate_embeddings(const std::vector<std::string>& inputs) const;

  const ValidatorConfig& config() const { return cfg_; }
  void set_config(const ValidatorConfig& c) { cfg_ = c; }

 private:
  ValidationResult check_sampling(size_t max_tokens, float temperature, float top_p) const;
  ValidatorConfig cfg_;
};

}  // namespace xgs
