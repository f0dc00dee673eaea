// Exceptions of the host API (include/mscclpp/errors.hpp:12-94): ErrorCode, the BaseError hierarchy
// and errorToString, with the reference's class names and messages, so a caller's catch clauses
// (`catch (const mscclpp::BaseError&)`, `mscclpp::Error`, `mscclpp::SysError`, `mscclpp::CudaError`)
// compile and match.  On this build a failed HIP runtime call surfaces as CudaError carrying the
// hipError_t (the reference's name for "a GPU runtime call failed", src/core/errors.cc:50-52);
// CuError and IbError exist for the catch clauses only (no driver-API or ibverbs path here).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace mscclpp_amd {

enum class ErrorCode { SystemError, InternalError, RemoteError, InvalidUsage, Timeout, Aborted, ExecutorError };

// errors.cc:12-29 (RemoteError, which the reference's switch omits, is named too)
inline std::string errorToString(ErrorCode error) {
  switch (error) {
    case ErrorCode::SystemError: return "SystemError";
    case ErrorCode::InternalError: return "InternalError";
    case ErrorCode::RemoteError: return "RemoteError";
    case ErrorCode::InvalidUsage: return "InvalidUsage";
    case ErrorCode::Timeout: return "Timeout";
    case ErrorCode::Aborted: return "Aborted";
    case ErrorCode::ExecutorError: return "ExecutorError";
  }
  return "UnknownError";
}

class BaseError : public std::runtime_error {
 public:
  BaseError(const std::string& message, int errorCode) : std::runtime_error(""), message_(message), errorCode_(errorCode) {}
  explicit BaseError(int errorCode) : std::runtime_error(""), errorCode_(errorCode) {}
  virtual ~BaseError() = default;
  int getErrorCode() const { return errorCode_; }
  const char* what() const noexcept override { return message_.c_str(); }

 protected:
  std::string message_;
  int errorCode_;
};

// errors.cc:38-44: the message carries the code's name
class Error : public BaseError {
 public:
  Error(const std::string& message, ErrorCode errorCode) : BaseError(static_cast<int>(errorCode)) {
    message_ = message + " (mscclpp failure: " + errorToString(errorCode) + ")";
  }
  virtual ~Error() = default;
  ErrorCode getErrorCode() const { return static_cast<ErrorCode>(errorCode_); }
};

class SysError : public BaseError {
 public:
  SysError(const std::string& message, int errorCode) : BaseError(errorCode) {
    message_ = message + " (System failure: " + std::strerror(errorCode) + ")";
  }
  virtual ~SysError() = default;
};

class CudaError : public BaseError {
 public:
  CudaError(const std::string& message, int errorCode) : BaseError(errorCode) {
    message_ = message + " (Cuda failure: " + hipGetErrorString(static_cast<hipError_t>(errorCode)) + ")";
  }
  virtual ~CudaError() = default;
};

class CuError : public BaseError {
 public:
  CuError(const std::string& message, int errorCode) : BaseError(errorCode) {
    message_ = message + " (Cu failure: " + hipGetErrorString(static_cast<hipError_t>(errorCode)) + ")";
  }
  virtual ~CuError() = default;
};

class IbError : public BaseError {
 public:
  IbError(const std::string& message, int errorCode) : BaseError(errorCode) {
    message_ = message + " (Ib failure: " + std::strerror(errorCode) + ")";
  }
  virtual ~IbError() = default;
};

}  // namespace mscclpp_amd
