# In-cluster conformance run of the e2e suite (config/conformance, `make conformance-run`):
# the controller image plus pytest and the e2e/ package — test tooling stays out of the
# production image.
ARG MANAGER_IMAGE=quay.io/opendatahub/odh-kubeflow-amd:main
FROM ${MANAGER_IMAGE}
USER 0
RUN pip install --no-cache-dir pytest
COPY e2e /opt/odh-kubeflow-amd/e2e
USER 65532:65532
WORKDIR /opt/odh-kubeflow-amd
ENTRYPOINT []
