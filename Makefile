# Developer targets (the reference's kf/Makefile and odh/Makefile counterparts).
PYTHON ?= python3
IMG ?= quay.io/opendatahub/odh-kubeflow-amd:$(shell cat releasing/VERSION)
PROBE_IMG ?= quay.io/opendatahub/odh-kubeflow-amd-gpu-probe:$(shell cat releasing/VERSION)
CONFORMANCE_IMG ?= quay.io/opendatahub/odh-kubeflow-amd-conformance:$(shell cat releasing/VERSION)
NOTEBOOK_IMG ?= quay.io/opendatahub/workbench-rocm-pytorch:latest
GPU_ARCH ?= gfx950

.PHONY: build test test-matrix test-native test-gpu e2e e2e-test conformance-run conformance-report conformance-clean coverage bench bench-8 manifests deploy deploy-sharded undeploy lint license-check docker-build docker-build-probe docker-build-conformance docker-push docker-build-notebook

build:  ## hipcc --offload-arch=$(GPU_ARCH) kernels, host C++ telemetry/objcore, native apiserver (in-tree)
	ODH_GPU_ARCH=$(GPU_ARCH) $(PYTHON) -m odh_kubeflow_amd.ops.build

test: build  ## CPU suite against the in-process store (envtest analogue)
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-matrix: build  ## the odh suites with SET_PIPELINE_RBAC=false and =true (odh/Makefile:106-115)
	ODH_TEST_SET_PIPELINE_RBAC=false $(PYTHON) -m pytest tests/test_odh_controller.py tests/test_odh_controller_scenarios.py -q
	ODH_TEST_SET_PIPELINE_RBAC=true $(PYTHON) -m pytest tests/test_odh_controller.py tests/test_odh_controller_scenarios.py -q

test-native: build  ## the same suite over the native C++ apiserver (REST + watch + HTTPS admission)
	ODH_CLUSTER_TRANSPORT=native $(PYTHON) -m pytest tests -q -m "not gpu"

test-gpu: build  ## HIP kernels vs fp32 torch on an MI355X
	$(PYTHON) -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread

e2e: build  ## separate apiserver / kf / odh / node-agent processes (reference e2e sequence)
	$(PYTHON) -m pytest tests/test_processes_e2e.py -q

# the reference's `make e2e-test` (odh/Makefile:192-197): against the cluster in $(KUBECONFIG)
# after `make deploy`, or — with no kubeconfig — against the dev stack as local processes.
# E2E_TEST_FLAGS e.g. "--nb-namespace e2e-notebook-controller --skip-deletion"
E2E_TEST_FLAGS ?=
e2e-test: build  ## e2e suite (e2e/): deployed overlay if KUBECONFIG is set, else local processes
	$(PYTHON) -m pytest e2e -v $(if $(KUBECONFIG),--kubeconfig $(KUBECONFIG)) $(E2E_TEST_FLAGS)

# in-cluster conformance run of the e2e suite (the reference's conformance/ Makefile flow):
# setup, the test pod, wait for its done file, copy the report out
CONFORMANCE_NS ?= odh-kubeflow-amd-conformance
conformance-run:  ## run the e2e suite as a pod in the current cluster (config/conformance)
	kubectl apply -f config/conformance/setup.yaml
	kubectl apply -f config/conformance/e2e-conformance.yaml
conformance-report:  ## wait for the conformance pod and copy its JUnit report to /tmp/odh-conformance
	until kubectl exec notebook-conformance -n $(CONFORMANCE_NS) -- ls /tmp/odh-conformance/done; do sleep 30; done
	mkdir -p /tmp/odh-conformance
	kubectl cp $(CONFORMANCE_NS)/notebook-conformance:/tmp/odh-conformance/junit.xml /tmp/odh-conformance/junit.xml
	kubectl exec notebook-conformance -n $(CONFORMANCE_NS) -- cat /tmp/odh-conformance/exit_code
conformance-clean:
	kubectl delete -f config/conformance/e2e-conformance.yaml -f config/conformance/setup.yaml

# per-component line coverage with floors (the reference's codecov flags, .codecov.yml:19-32)
coverage: build  ## line coverage of the CPU suite per component (tools/coverage.py → coverage.json)
	$(PYTHON) tools/coverage.py --flag kf=78 --flag odh=85 --flag runtime=84 --flag apiserver=85

bench: build  ## headline benchmark on one MI355X
	$(PYTHON) bench.py

bench-8: build  ## one control-plane shard per MI355X of an 8-GPU node
	$(PYTHON) -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

manifests:  ## regenerate the kustomize tree under config/
	$(PYTHON) -m odh_kubeflow_amd.deploy.manifests --out config

OVERLAY ?= mi355x
deploy: manifests  ## kubectl apply an overlay (OVERLAY=mi355x|standalone|kubeflow|openshift): CRD, RBAC, managers, webhook, node agent
	kubectl apply -k config/overlays/$(OVERLAY)

deploy-sharded: manifests  ## kubectl apply the sharded MI355X overlay (one control-plane shard per GPU)
	kubectl apply -k config/overlays/mi355x-sharded

undeploy:
	kubectl delete -k config/overlays/$(OVERLAY) --ignore-not-found

lint:  ## static analysis: Python AST rules, secrets, rendered manifests, -Wall -Wextra -Werror native builds
	$(PYTHON) tools/lint.py

license-check:  ## runtime dependencies carry permissive licences (kf/third_party/check-license.sh)
	$(PYTHON) tools/licenses.py

docker-build:  ## controller / webhook / node-agent image (slim Python, host C++ only; no ROCm, no torch)
	docker build -f images/Dockerfile -t $(IMG) .

docker-build-probe:  ## MI355X start-up probe init-container image (ROCm runtime; kernels for $(GPU_ARCH))
	docker build -f images/probe.Dockerfile --build-arg GPU_ARCH=$(GPU_ARCH) -t $(PROBE_IMG) .

docker-build-conformance: docker-build  ## controller image + pytest + e2e/ (config/conformance)
	docker build -f images/conformance.Dockerfile --build-arg MANAGER_IMAGE=$(IMG) -t $(CONFORMANCE_IMG) .

docker-push:  ## push the controller / node-agent and probe images
	docker push $(IMG)
	docker push $(PROBE_IMG)

docker-build-notebook:  ## PyTorch-ROCm Jupyter workbench image the samples reference
	docker build -f images/notebook.Dockerfile -t $(NOTEBOOK_IMG) images
