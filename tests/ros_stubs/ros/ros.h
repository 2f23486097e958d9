// stub (syntax check only): the roscpp surface the node adapters use --
// NodeHandle parameters / topics / services, Time, and the ROS_* log macros.
#pragma once
#include <cstdio>
#include <string>

#include <boost/shared_ptr.hpp>

#define ROS_INFO(...) std::printf(__VA_ARGS__)
#define ROS_WARN(...) std::printf(__VA_ARGS__)
#define ROS_ERROR(...) std::printf(__VA_ARGS__)

namespace ros {

struct Duration {
  double sec = 0.0;
  double toSec() const { return sec; }
};

struct Time {
  double t = 0.0;
  static Time now() { return Time(); }
  Duration operator-(const Time& o) const { return Duration{t - o.t}; }
};

class Publisher {
 public:
  template <class M>
  void publish(const M&) const {}
  template <class M>
  void publish(const boost::shared_ptr<M>&) const {}
};

class Subscriber {};
class ServiceServer {};

class NodeHandle {
 public:
  bool getParam(const std::string&, std::string&) const { return true; }
  bool getParam(const std::string&, int&) const { return true; }
  bool getParam(const std::string&, float&) const { return true; }
  bool getParam(const std::string&, double&) const { return true; }
  bool getParam(const std::string&, bool&) const { return true; }
  template <class T>
  bool param(const std::string&, T& v, const T& d) const {
    v = d;
    return true;
  }
  template <class M>
  Publisher advertise(const std::string&, unsigned, bool latch = false) {
    (void)latch;
    return Publisher();
  }
  template <class M, class C>
  Subscriber subscribe(const std::string&, unsigned, void (C::*)(const boost::shared_ptr<const M>&),
                       C*) {
    return Subscriber();
  }
  template <class C, class Req, class Res>
  ServiceServer advertiseService(const std::string&, bool (C::*)(Req&, Res&), C*) {
    return ServiceServer();
  }
};

}  // namespace ros
