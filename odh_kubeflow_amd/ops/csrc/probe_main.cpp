// odh-gpu-probe: the notebook pod's MI355X start-up probe (init container entry point).
// Everything lives in probe_cli.cpp (odh_probe_cli), shared with `python -m odh_kubeflow_amd.ops.probe_main`.
extern "C" int odh_probe_cli(int argc, char** argv);

int main(int argc, char** argv) { return odh_probe_cli(argc, argv); }
