// Umbrella header, like hpipm-cpp/include/hpipm-cpp/hpipm-cpp.hpp.
#pragma once

#include "hpipm-cpp/ocp_qp.hpp"
#include "hpipm-cpp/ocp_qp_dim.hpp"
#include "hpipm-cpp/ocp_qp_ipm_solver.hpp"
#include "hpipm-cpp/ocp_qp_ipm_solver_settings.hpp"
#include "hpipm-cpp/ocp_qp_ipm_solver_statistics.hpp"
#include "hpipm-cpp/ocp_qp_solution.hpp"
