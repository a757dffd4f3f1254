"""Handles for every kind the controllers touch (``"apiVersion/Kind"`` strings)."""

POD = "v1/Pod"
SERVICE = "v1/Service"
SERVICE_ACCOUNT = "v1/ServiceAccount"
CONFIG_MAP = "v1/ConfigMap"
SECRET = "v1/Secret"
EVENT = "v1/Event"
NAMESPACE = "v1/Namespace"
NODE = "v1/Node"
STATEFUL_SET = "apps/v1/StatefulSet"
DEPLOYMENT = "apps/v1/Deployment"
DAEMON_SET = "apps/v1/DaemonSet"
NETWORK_POLICY = "networking.k8s.io/v1/NetworkPolicy"
ROLE = "rbac.authorization.k8s.io/v1/Role"
ROLE_BINDING = "rbac.authorization.k8s.io/v1/RoleBinding"
CLUSTER_ROLE = "rbac.authorization.k8s.io/v1/ClusterRole"
CLUSTER_ROLE_BINDING = "rbac.authorization.k8s.io/v1/ClusterRoleBinding"
LEASE = "coordination.k8s.io/v1/Lease"
MUTATING_WEBHOOK_CONFIGURATION = "admissionregistration.k8s.io/v1/MutatingWebhookConfiguration"
CRD = "apiextensions.k8s.io/v1/CustomResourceDefinition"
CSR = "certificates.k8s.io/v1/CertificateSigningRequest"

NOTEBOOK_V1 = "kubeflow.org/v1/Notebook"
NOTEBOOK_V1ALPHA1 = "kubeflow.org/v1alpha1/Notebook"
NOTEBOOK_V1BETA1 = "kubeflow.org/v1beta1/Notebook"
NOTEBOOK = NOTEBOOK_V1

VIRTUAL_SERVICE = "networking.istio.io/v1alpha3/VirtualService"
HTTP_ROUTE = "gateway.networking.k8s.io/v1/HTTPRoute"
GATEWAY = "gateway.networking.k8s.io/v1/Gateway"
REFERENCE_GRANT = "gateway.networking.k8s.io/v1beta1/ReferenceGrant"
IMAGE_STREAM = "image.openshift.io/v1/ImageStream"
PROXY = "config.openshift.io/v1/Proxy"
ROUTE = "route.openshift.io/v1/Route"
OAUTH_CLIENT = "oauth.openshift.io/v1/OAuthClient"
DSPA = "datasciencepipelinesapplications.opendatahub.io/v1/DataSciencePipelinesApplication"


def split(kind_ref: str):
    api_version, _, kind = kind_ref.rpartition("/")
    return api_version, kind
