// POMDP node class of the catkin package, rebuilt on libpp2_hip.so.
//
// Replaces include/path_planning_2d/pomdp_path_planning_2d.h of the reference
// (class at :37-87).  Same public interface, parameters, topics and services;
// the online tree (SearchTree* search_tree, :80) and the model/FIB/PBVI device
// globals become one pp2_ctx (the grid's device state) and one pp2_planner
// (the QV-tree), both owned by the node.  Syntax-checked with both adapters
// (tests/test_ros_adapters.py); see ros/README.md.
#ifndef POMDP_PATH_PLANNING_2D_H
#define POMDP_PATH_PLANNING_2D_H

#include <std_srvs/Trigger.h>

#include <pp2.h>

#include "path_planning_2d_base.h"

namespace path_planning_2d {

class PomdpPathPlanning2d : public PathPlanning2dBase {
 public:
  typedef boost::shared_ptr<PomdpPathPlanning2d> Ptr;
  typedef boost::shared_ptr<const PomdpPathPlanning2d> ConstPtr;

  explicit PomdpPathPlanning2d(ros::NodeHandle& n);
  PomdpPathPlanning2d(const PomdpPathPlanning2d&) = delete;
  PomdpPathPlanning2d operator=(const PomdpPathPlanning2d&) = delete;
  ~PomdpPathPlanning2d();

  virtual bool initialize();

 private:
  virtual bool loadParameters();
  virtual bool createRosIO();
  virtual void beliefCallback(const dummy_simulator::BeliefConstPtr& belief);
  virtual void loadMapFromFile();

  bool saveDataCallback(std_srvs::Trigger::Request& req, std_srvs::Trigger::Response& res);
  bool resetSearchTreeCallback(std_srvs::Trigger::Request& req,
                               std_srvs::Trigger::Response& res);

  // Offline solutions (model, FIB upper bound, PBVI lower bound) from files
  // instead of solving them at start-up (launch parameter read_data_from_file).
  bool read_from_file = false;
  int32_t max_search_tree_depth = 5;
  int32_t max_online_iteration = 5;

  pp2_ctx* ctx_ = nullptr;          // model, FIB and PBVI data on the GPU
  pp2_planner* planner_ = nullptr;  // the online QV-tree

  ros::ServiceServer save_data_server;
  ros::ServiceServer reset_search_tree_server;
};

typedef PomdpPathPlanning2d::Ptr PomdpPathPlanning2dPtr;
typedef PomdpPathPlanning2d::ConstPtr PomdpPathPlanning2dConstPtr;
}  // namespace path_planning_2d

#endif
