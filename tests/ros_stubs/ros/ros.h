// stand-in roscpp (tests only): the surface the node adapters use --
// NodeHandle parameters / topics / services, Time, the ROS_* log macros --
// with a working in-process transport, so tests/ros_stubs/run_node.cpp can
// drive a node: parameters come from ros::stub::params(), publish() appends to
// ros::stub::published<M>()[topic], subscribe() / advertiseService() register
// callables the driver invokes.  Signatures follow roscpp.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include <boost/shared_ptr.hpp>

#define ROS_INFO(...) (std::printf(__VA_ARGS__), std::printf("\n"))
#define ROS_WARN(...) (std::printf(__VA_ARGS__), std::printf("\n"))
#define ROS_ERROR(...) (std::fprintf(stderr, __VA_ARGS__), std::fprintf(stderr, "\n"))

namespace ros {

inline void init(int&, char**, const std::string&) {}
inline void spin() {}

struct Duration {
  double sec = 0.0;
  double toSec() const { return sec; }
};

struct Time {
  double t = 0.0;
  static Time now() {
    using namespace std::chrono;
    return Time{duration<double>(steady_clock::now().time_since_epoch()).count()};
  }
  Duration operator-(const Time& o) const { return Duration{t - o.t}; }
};

namespace stub {
inline std::map<std::string, std::string>& params() {
  static std::map<std::string, std::string> m;
  return m;
}
template <class M>
std::map<std::string, std::vector<M>>& published() {
  static std::map<std::string, std::vector<M>> m;
  return m;
}
template <class M>
std::map<std::string, std::function<void(const boost::shared_ptr<const M>&)>>& subscribers() {
  static std::map<std::string, std::function<void(const boost::shared_ptr<const M>&)>> m;
  return m;
}
template <class Req, class Res>
std::map<std::string, std::function<bool(Req&, Res&)>>& services() {
  static std::map<std::string, std::function<bool(Req&, Res&)>> m;
  return m;
}
inline bool parse(const std::string& s, std::string& v) { v = s; return true; }
inline bool parse(const std::string& s, int& v) { v = std::atoi(s.c_str()); return true; }
inline bool parse(const std::string& s, float& v) { v = std::strtof(s.c_str(), nullptr); return true; }
inline bool parse(const std::string& s, double& v) { v = std::strtod(s.c_str(), nullptr); return true; }
inline bool parse(const std::string& s, bool& v) {
  v = s == "true" || s == "1";
  return true;
}
}  // namespace stub

class Publisher {
 public:
  Publisher() = default;
  explicit Publisher(const std::string& topic) : topic_(topic) {}
  template <class M>
  void publish(const M& m) const {
    stub::published<M>()[topic_].push_back(m);
  }
  template <class M>
  void publish(const boost::shared_ptr<M>& m) const {
    publish(*m);
  }

 private:
  std::string topic_;
};

class Subscriber {};
class ServiceServer {};

class NodeHandle {
 public:
  NodeHandle() = default;
  explicit NodeHandle(const std::string&) {}
  template <class T>
  bool getParam(const std::string& key, T& v) const {
    const auto it = stub::params().find(key);
    return it != stub::params().end() && stub::parse(it->second, v);
  }
  template <class T>
  bool param(const std::string& key, T& v, const T& d) const {
    if (!getParam(key, v)) v = d;
    return true;
  }
  template <class M>
  Publisher advertise(const std::string& topic, unsigned, bool latch = false) {
    (void)latch;
    return Publisher(topic);
  }
  template <class M, class C>
  Subscriber subscribe(const std::string& topic, unsigned,
                       void (C::*fp)(const boost::shared_ptr<const M>&), C* obj) {
    stub::subscribers<M>()[topic] = [obj, fp](const boost::shared_ptr<const M>& m) {
      (obj->*fp)(m);
    };
    return Subscriber();
  }
  template <class C, class Req, class Res>
  ServiceServer advertiseService(const std::string& name, bool (C::*fp)(Req&, Res&), C* obj) {
    stub::services<Req, Res>()[name] = [obj, fp](Req& q, Res& s) { return (obj->*fp)(q, s); };
    return ServiceServer();
  }
};

}  // namespace ros
