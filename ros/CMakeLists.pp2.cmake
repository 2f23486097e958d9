# Drop-in for path_planning_2d/CMakeLists.txt of the reference (the CUDA part,
# :30-40 and the cuda_add_executable targets :105-140): include this file
# after catkin_package() in place of find_package(CUDA) and the two CUDA node
# targets.  PP2_ROOT points at this repository; libpp2_hip.so is built by
# `make -C path_planning_2d_amd/csrc` (hipcc, gfx950; HIP runtime + RCCL).
#
#   include(/path/to/this/repo/ros/CMakeLists.pp2.cmake)
#
# The adapter sources below replace src/pomdp/path_planning_2d.cu and
# src/mdp/path_planning_2d.cu; ros/include/ comes first on the include path
# so its pomdp_path_planning_2d.h (pp2_ctx / pp2_planner members instead of
# SearchTree*) shadows the reference header.  The A* node's target is
# unchanged.
get_filename_component(PP2_ROOT ${CMAKE_CURRENT_LIST_DIR}/.. ABSOLUTE)

add_library(pp2_hip SHARED IMPORTED)
set_target_properties(pp2_hip PROPERTIES
  IMPORTED_LOCATION ${PP2_ROOT}/path_planning_2d_amd/libpp2_hip.so
  INTERFACE_INCLUDE_DIRECTORIES ${PP2_ROOT}/include)

find_package(OpenCV REQUIRED)

add_executable(pomdp_path_planning_2d_node
  src/pomdp/path_planning_2d_node.cpp
  ${PP2_ROOT}/ros/src/pomdp/path_planning_2d_pp2.cpp)
target_include_directories(pomdp_path_planning_2d_node BEFORE PRIVATE ${PP2_ROOT}/ros/include)
target_link_libraries(pomdp_path_planning_2d_node pp2_hip ${catkin_LIBRARIES} ${OpenCV_LIBRARIES})
add_dependencies(pomdp_path_planning_2d_node ${catkin_EXPORTED_TARGETS})

add_executable(mdp_path_planning_2d_node
  src/mdp/path_planning_2d_node.cpp
  ${PP2_ROOT}/ros/src/mdp/path_planning_2d_pp2.cpp)
target_link_libraries(mdp_path_planning_2d_node pp2_hip ${catkin_LIBRARIES} ${OpenCV_LIBRARIES})
add_dependencies(mdp_path_planning_2d_node ${catkin_EXPORTED_TARGETS})
