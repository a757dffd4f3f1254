"""Names shared by the ODH reconciler and the mutating webhook.

Every string here is part of the observable protocol of the reference
(``odh/controllers/notebook_controller.go:55-79``, ``notebook_webhook.go:74-96``,
``notebook_network.go:35-40``, ``notebook_kube_rbac_auth.go:38-43``,
``notebook_route.go:36-48``, ``notebook_referencegrant.go:33``,
``notebook_runtime.go:20-24``, ``notebook_dspa_secret.go:38-47``,
``notebook_feast_config.go:27-31``, ``notebook_oauth.go:31``) and must not change.
"""

from ...models.notebook import STOP_ANNOTATION  # noqa: F401  (culler.STOP_ANNOTATION)

# annotations
ANNOTATION_INJECT_AUTH = "notebooks.opendatahub.io/inject-auth"
ANNOTATION_VALUE_RECONCILIATION_LOCK = "odh-notebook-controller-lock"
ANNOTATION_AUTH_SIDECAR_CPU_REQUEST = "notebooks.opendatahub.io/auth-sidecar-cpu-request"
ANNOTATION_AUTH_SIDECAR_MEMORY_REQUEST = "notebooks.opendatahub.io/auth-sidecar-memory-request"
ANNOTATION_AUTH_SIDECAR_CPU_LIMIT = "notebooks.opendatahub.io/auth-sidecar-cpu-limit"
ANNOTATION_AUTH_SIDECAR_MEMORY_LIMIT = "notebooks.opendatahub.io/auth-sidecar-memory-limit"
DEFAULT_AUTH_SIDECAR_CPU_REQUEST = "100m"
DEFAULT_AUTH_SIDECAR_MEMORY_REQUEST = "64Mi"
DEFAULT_AUTH_SIDECAR_CPU_LIMIT = "100m"
DEFAULT_AUTH_SIDECAR_MEMORY_LIMIT = "64Mi"
ANNOTATION_UPDATE_PENDING = "notebooks.opendatahub.io/update-pending"
ANNOTATION_NOTEBOOK_RESTART = "notebooks.opendatahub.io/notebook-restart"
WORKBENCH_IMAGE_NAMESPACE_ANNOTATION = "opendatahub.io/workbench-image-namespace"
LAST_IMAGE_SELECTION_ANNOTATION = "notebooks.opendatahub.io/last-image-selection"

# finalizers
HTTPROUTE_FINALIZER = "notebook.opendatahub.io/httproute-cleanup"
REFERENCEGRANT_FINALIZER = "notebook.opendatahub.io/referencegrant-cleanup"
KUBE_RBAC_PROXY_FINALIZER = "notebook.opendatahub.io/kube-rbac-proxy-cleanup"
OAUTH_CLIENT_FINALIZER = "notebook-oauth-client-finalizer.opendatahub.io"

# trusted CA bundle
ODH_CONFIGMAP_NAME = "odh-trusted-ca-bundle"
SELF_SIGNED_CONFIGMAP_NAME = "kube-root-ca.crt"
SERVICE_CA_CONFIGMAP_NAME = "openshift-service-ca.crt"
WORKBENCH_CA_CONFIGMAP_NAME = "workbench-trusted-ca-bundle"
CA_VOLUME_NAME = "trusted-ca"
CA_MOUNT_PATH = "/etc/pki/tls/custom-certs/ca-bundle.crt"
CA_KEY = "ca-bundle.crt"
CA_ENV_VARS = ("PIP_CERT", "REQUESTS_CA_BUNDLE", "SSL_CERT_FILE", "PIPELINES_SSL_SA_CERTS",
               "KF_PIPELINES_SSL_SA_CERTS", "GIT_SSL_CAINFO")

# ports / network
NOTEBOOK_PORT = 8888
KUBE_RBAC_PROXY_PORT = 8443
KUBE_RBAC_PROXY_HEALTH_PORT = 8444
KUBE_RBAC_PROXY_NP_SUFFIX = "-kube-rbac-proxy-np"
CTRL_NP_SUFFIX = "-ctrl-np"

# kube-rbac-proxy
CONTAINER_NAME_KUBE_RBAC_PROXY = "kube-rbac-proxy"
KUBE_RBAC_PROXY_CONFIG_VOLUME = "kube-rbac-proxy-config"
KUBE_RBAC_PROXY_CONFIG_MOUNT_PATH = "/etc/kube-rbac-proxy"
KUBE_RBAC_PROXY_CONFIG_FILE = "config-file.yaml"
KUBE_RBAC_PROXY_TLS_VOLUME = "kube-rbac-proxy-tls-certificates"
KUBE_RBAC_PROXY_TLS_MOUNT_PATH = "/etc/tls/private"
KUBE_RBAC_PROXY_TLS_SECRET_SUFFIX = "-kube-rbac-proxy-tls"
KUBE_RBAC_PROXY_SERVICE_PORT_NAME = "kube-rbac-proxy"
KUBE_RBAC_PROXY_CONFIG_SUFFIX = "-kube-rbac-proxy-config"
KUBE_RBAC_PROXY_SERVICE_SUFFIX = "-kube-rbac-proxy"

# gateway api
HTTPROUTE_SUBDOMAIN_MAX_LEN = 63
DEFAULT_GATEWAY_NAME = "data-science-gateway"
DEFAULT_GATEWAY_NAMESPACE = "openshift-ingress"
REFERENCE_GRANT_NAME = "notebook-httproute-access"

# pipelines
RUNTIME_IMAGES_CONFIGMAP = "pipeline-runtime-images"
RUNTIME_IMAGES_MOUNT_PATH = "/opt/app-root/pipeline-runtimes/"
RUNTIME_IMAGES_VOLUME = "runtime-images"
RUNTIME_IMAGE_LABEL = "opendatahub.io/runtime-image"
RUNTIME_IMAGE_METADATA_ANNOTATION = "opendatahub.io/runtime-image-metadata"
ELYRA_SECRET_NAME = "ds-pipeline-config"
ELYRA_MOUNT_PATH = "/opt/app-root/runtimes"
ELYRA_VOLUME_NAME = "elyra-dsp-details"
DSPA_INSTANCE_NAME = "dspa"
DSPA_ROLE_NAME = "ds-pipeline-user-access-dspa"
MANAGED_BY_KEY = "opendatahub.io/managed-by"
MANAGED_BY_VALUE = "workbenches"

# feast
FEAST_CONFIGMAP_SUFFIX = "-feast-config"
FEAST_VOLUME_NAME = "odh-feast-config"
FEAST_MOUNT_PATH = "/opt/app-root/src/feast-config"
FEAST_LABEL = "opendatahub.io/feast-integration"

# tracing span events (notebook_webhook.go:89-90)
IMAGE_STREAM_NOT_FOUND_EVENT = "imagestream-not-found"
IMAGE_STREAM_TAG_NOT_FOUND_EVENT = "imagestream-tag-not-found"
INTERNAL_REGISTRY = "image-registry.openshift-image-registry.svc:5000"
