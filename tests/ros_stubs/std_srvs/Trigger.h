// stand-in (tests only): std_srvs/Trigger
#pragma once
#include <string>
namespace std_srvs {
struct Trigger {
  struct Request {};
  struct Response {
    bool success = false;
    std::string message;
  };
};
}  // namespace std_srvs
