// odh-gpu-probe: the notebook pod's MI355X start-up probe (init container entry point).
// Everything lives in probe_cli.cpp (odh_probe_cli), shared with `python -m odh_kubeflow_amd.ops.probe_main`.
#include <cstdio>
#include <cstdlib>

extern "C" int odh_probe_cli(int argc, char** argv);

int main(int argc, char** argv) {
  const int rc = odh_probe_cli(argc, argv);
  // the verdict is written and flushed: leave without the HIP runtime's exit-time teardown
  // (the kernel driver reclaims the process's GPU state) — it only delays the notebook's start
  std::fflush(nullptr);
  std::_Exit(rc);
}
