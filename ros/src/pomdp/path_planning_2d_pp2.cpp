// PomdpPathPlanning2d on libpp2_hip.so: replaces src/pomdp/path_planning_2d.cu
// of the reference (class body :61-282) in the catkin package.  The node
// main (src/pomdp/path_planning_2d_node.cpp), launch files, parameters,
// topics ("belief" in, "control" out) and services ("save_data",
// "reset_search_tree") are unchanged; every CUDA call is a pp2.h call.
//
// Syntax-checked here (tests/test_ros_adapters.py: g++ -fsyntax-only -Werror
// against the stand-in ROS / OpenCV headers of tests/ros_stubs/); the image
// has no ROS, OpenCV or Boost to link it.  tests/test_abi.py compiles the same
// pp2.h call sequence in plain C (examples/pp2_node_demo.c) and
// tests/test_gpu_planner.py runs it.
#include <cstdio>
#include <vector>

#include <opencv2/core/core.hpp>
#include <opencv2/highgui/highgui.hpp>

#include <std_msgs/Byte.h>

#include <path_planning_2d/pomdp_path_planning_2d.h>

namespace path_planning_2d {

namespace {

// Belief set size of the reference's PBVI (src/pomdp/path_planning_2d.cu:122).
constexpr uint32_t kBeliefSetSize = 500;

bool pp2_ok(int status, const char* what) {
  if (status == PP2_OK) return true;
  ROS_ERROR("%s failed (%s): %s", what, pp2_status_string(status), pp2_last_error());
  return false;
}

}  // namespace

PomdpPathPlanning2d::PomdpPathPlanning2d(ros::NodeHandle& n) : PathPlanning2dBase(n) {}

PomdpPathPlanning2d::~PomdpPathPlanning2d() {
  if (planner_) pp2_planner_destroy(planner_);
  if (ctx_) pp2_destroy(ctx_);
  free(grid_map);
  if (planning_time_fid) fclose(planning_time_fid);
}

bool PomdpPathPlanning2d::loadParameters() {
  // required, in the reference's order; the frame ids have defaults
  const bool ok = nh.getParam("map_path", map_path) && nh.getParam("goal_x", goal[0]) &&
                  nh.getParam("goal_y", goal[1]) &&
                  nh.getParam("discount_factor", discount_factor) &&
                  nh.getParam("map_resolution", map_resolution) &&
                  nh.getParam("read_data_from_file", read_from_file) &&
                  nh.getParam("max_search_tree_depth", max_search_tree_depth) &&
                  nh.getParam("max_online_iteration", max_online_iteration);
  nh.param<std::string>("fixed_frame_id", fixed_frame_id, "map");
  nh.param<std::string>("robot_frame_id", robot_frame_id, "robot");
  return ok;
}

// Occupancy grid from the map image: 1 where the grey level is <= 250
// (cv::threshold(img, out, 250, 1, THRESH_BINARY_INV) of the reference).
void PomdpPathPlanning2d::loadMapFromFile() {
  const cv::Mat img = cv::imread(map_path, cv::IMREAD_GRAYSCALE);
  map_height = img.rows;
  map_width = img.cols;
  grid_map = static_cast<uint8_t*>(malloc((size_t)map_height * map_width));
  for (uint32_t y = 0; y < map_height; ++y) {
    const uint8_t* row = img.ptr<uint8_t>(y);
    for (uint32_t x = 0; x < map_width; ++x) grid_map[(size_t)y * map_width + x] = row[x] <= 250;
  }
}

bool PomdpPathPlanning2d::initialize() {
  if (!loadParameters()) {
    ROS_WARN("Cannot load all required parameters...");
    return false;
  }
  loadMapFromFile();
  if (grid_map[(size_t)goal[1] * map_width + goal[0]]) {
    ROS_ERROR("The assigned goal (%d %d) is at a occupied cell...", goal[0], goal[1]);
    return false;
  }
  // uniform initial belief over the free cells, fp32 as the reference builds it
  const size_t hw = (size_t)map_height * map_width;
  float n_free = 0.0f;
  for (size_t i = 0; i < hw; ++i) n_free += 1.0f - grid_map[i];
  std::vector<float> b0(hw);
  for (size_t i = 0; i < hw; ++i) b0[i] = (1.0f - grid_map[i]) / n_free;

  if (!pp2_ok(pp2_create(&ctx_, /*device=*/0, map_height, map_width, grid_map, goal[0], goal[1],
                         discount_factor),
              "pp2_create"))
    return false;
  uint64_t rand_draws = 0;  // glibc rand() calls PBVI's belief set consumed
  if (!read_from_file) {
    int fib_sweeps = 0;
    float fib_norm = 0.0f;
    if (!pp2_ok(pp2_model_generate(ctx_), "model generation") ||
        !pp2_ok(pp2_fib_solve(ctx_, 0, &fib_sweeps, &fib_norm), "FIB") ||
        !pp2_ok(pp2_pbvi_solve(ctx_, b0.data(), kBeliefSetSize, /*rand_seed=*/1, &rand_draws),
                "PBVI"))
      return false;
    ROS_INFO("model, FIB (%d sweeps) and PBVI (%u beliefs) solved on the GPU", fib_sweeps,
             kBeliefSetSize);
  } else {
    // model_data_*, fib_*, pbvi_* in the working directory (saveDataCallback)
    if (!pp2_ok(pp2_model_load(ctx_, "."), "loading model data") ||
        !pp2_ok(pp2_fib_load(ctx_, "."), "loading FIB data") ||
        !pp2_ok(pp2_pbvi_load(ctx_, ".", kBeliefSetSize), "loading PBVI data"))
      return false;
  }
  pp2_planner_params prm;
  pp2_planner_default_params(&prm);
  prm.max_search_tree_depth = max_search_tree_depth;
  prm.max_online_iteration = max_online_iteration;
  prm.lower_bound_mode = 1;     // leaf lower bounds from the PBVI alphas
  prm.rand_skip = rand_draws;   // the tree's rand() stream continues PBVI's
  // (the default, stated): every grid-wide sum gives the reference's x-ordered
  // fp32 host result, so the published actions equal the reference's bit for bit
  prm.reference_order = 1;
  if (!pp2_ok(pp2_planner_create(&planner_, ctx_, &prm), "planner")) return false;

  if (!createRosIO()) {
    ROS_WARN("Cannot load all ROS I/O");
    return false;
  }
  planning_time_fid = fopen("planning_time", "a+");
  return true;
}

bool PomdpPathPlanning2d::createRosIO() {
  control_pub = nh.advertise<std_msgs::Byte>("control", 1);
  belief_sub = nh.subscribe("belief", 1, &PomdpPathPlanning2d::beliefCallback, this);
  save_data_server =
      nh.advertiseService("save_data", &PomdpPathPlanning2d::saveDataCallback, this);
  reset_search_tree_server = nh.advertiseService(
      "reset_search_tree", &PomdpPathPlanning2d::resetSearchTreeCallback, this);
  return true;
}

// One plan step: the first message (or the first after reset_search_tree)
// roots a new tree at its belief, later ones re-root by (action,
// observation); expansions and the action choice run inside pp2_planner_step.
void PomdpPathPlanning2d::beliefCallback(const dummy_simulator::BeliefConstPtr& msg) {
  uint8_t z = 0;
  for (int bit = 3; bit >= 0; --bit) z = (uint8_t)(2 * z + msg->measurement[bit]);
  const ros::Time t0 = ros::Time::now();
  uint8_t next_action = 0;
  float next_value = 0.0f;
  if (!pp2_ok(pp2_planner_step(planner_, msg->action, z, msg->belief.data(), &next_action,
                               &next_value),
              "plan step"))
    return;
  pp2_tree_info info;
  if (pp2_planner_info(planner_, &info) == PP2_OK)
    printf("planning time: %f\nSearch tree depth: %u\n", (ros::Time::now() - t0).toSec(),
           info.depth);
  std_msgs::BytePtr out(new std_msgs::Byte);
  out->data = next_action;
  control_pub.publish(out);
}

bool PomdpPathPlanning2d::saveDataCallback(std_srvs::Trigger::Request&,
                                           std_srvs::Trigger::Response& res) {
  // the reference's text files: model_data_*, fib_alphas/actions, pbvi_alphas/actions
  res.success = pp2_ok(pp2_model_save(ctx_, "."), "saving model data") &&
                pp2_ok(pp2_fib_save(ctx_, "."), "saving FIB data") &&
                pp2_ok(pp2_pbvi_save(ctx_, "."), "saving PBVI data");
  return true;
}

bool PomdpPathPlanning2d::resetSearchTreeCallback(std_srvs::Trigger::Request&,
                                                  std_srvs::Trigger::Response&) {
  pp2_planner_reset(planner_);
  return true;
}

}  // namespace path_planning_2d
