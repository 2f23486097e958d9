// stand-in (tests only): boost::shared_ptr as the adapters use it
#pragma once
#include <memory>
namespace boost {
using std::shared_ptr;
}
