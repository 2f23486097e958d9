// stand-in (tests only): std_msgs/Byte
#pragma once
#include <cstdint>
#include <boost/shared_ptr.hpp>
namespace std_msgs {
struct Byte {
  int8_t data = 0;
};
typedef boost::shared_ptr<Byte> BytePtr;
}  // namespace std_msgs
