"""Resource names, annotation keys and constants (wire-compatible with the reference).

Reference: pkg/types/types.go:7-21, pkg/dealer/type.go:5-9, pkg/controller/node.go:18-24.
"""
from __future__ import annotations

# --- reference contract (kept byte-identical) -------------------------------------
RESOURCE_GPU_PERCENT = "nano-gpu/gpu-percent"          # types.go:9
GPU_PERCENT_EACH_CARD = 100                            # types.go:10
GPU_ASSUME = "nano-gpu/assume"                         # types.go:12-14 (annotation AND label)
ANNOTATION_GPU_ASSUME = GPU_ASSUME
LABEL_GPU_ASSUME = GPU_ASSUME
ANNOTATION_CONTAINER_FMT = "nano-gpu/container-{}"     # types.go:15 ("nano-gpu/container-%s")
NODE_NAME_FIELD = "spec.nodeName"                      # types.go:8
PRIORITY_BINPACK = "binpack"                           # types.go:19
PRIORITY_SPREAD = "spread"                             # types.go:20
NOT_NEED_GPU = -1                                      # allocate.go:15
LOAD_TOTAL = 2                                         # allocate.go:16
SCORE_MIN = 0                                          # rater.go:12
SCORE_MAX = 100                                        # rater.go:13
VERSION = "0.1.0"                                      # routes.go:30 (compat /version)
FRAMEWORK_VERSION = "0.1.0-mi355x"

GPU_CORE_USAGE_METRIC = "gpu_core_usage_avg"           # type.go:7
GPU_MEMORY_USAGE_METRIC = "gpu_memory_usage_avg"       # type.go:8
EXTENDER_ACTIVE_PERIOD_S = 300.0                       # type.go:6 (5 minutes)
LEGACY_GPU_NODE_LABEL = ("nvidia-device-enable", "enable")  # controller/node.go:153-158

# --- MI355X-native additions --------------------------------------------------------
PRIORITY_RANDOM = "random"        # promised by reference README.md:14, absent in its code
PRIORITY_FIRSTFIT = "firstfit"    # reference SampleRater (rater.go:21-50), test-only there
POLICIES = (PRIORITY_BINPACK, PRIORITY_SPREAD, PRIORITY_RANDOM, PRIORITY_FIRSTFIT)
# Priorities answer the nominated node this many raw points above every other fitting node.
# kube-scheduler adds 10 x (extender score x weight) to its own plugins' sum; the default plugins
# that differ between GPU nodes (LeastAllocated, BalancedAllocation, PodTopologySpread x 2,
# ImageLocality, InterPodAffinity, NodeAffinity, TaintToleration) span at most ~800 points, so
# 100 raw points (1,000) keep the pod on its nomination. 0 answers the raw scores (reference).
PRIORITY_LEAD = 100
# kube-apiserver's --max-mutating-requests-inflight default: the native bind writer sizes its
# window under it (nanogpu.app.Config.writer_max_binds) and backs off on its 429s
API_MAX_MUTATING_INFLIGHT = 200

RESOURCE_GPU_MEMORY = "nano-gpu/gpu-memory"   # HBM MiB per container (288 GB / MI355X)
ANNOTATION_TOPOLOGY = "nano-gpu/topology"     # node: JSON from the node agent (topology.model)
ANNOTATION_RECONCILED = "nano-gpu/reconciled"   # pod: the agent rewrote its placement to what kubelet ran
ANNOTATION_CU_MASK_FMT = "nano-gpu/cu-mask-{}"  # pod: per-container CU mask chosen by the agent
ANNOTATION_ASSUME_TIME = "nano-gpu/assume-time"
ANNOTATION_SCHEDULER = "nano-gpu/scheduler"
# pod: "true" or a comma list of containers that stream HBM (memory-bound); native policies
# keep them apart from each other on a device (native/include/nanogpu/alloc.h kFlagMemBound)
ANNOTATION_MEMORY_BOUND = "nano-gpu/memory-bound"
FLAG_MEM_BOUND = 1
# Measured memory-boundness: a policy that polls this metric (HBM / memory-controller activity
# in [0, 1]) marks a device whose activity is at or above HBM_HOT_THRESHOLD as holding a
# streaming tenant (alloc.h Device::mem_hot), declared or not. It feeds only that mark, not the
# reference's load sum (RemainLoad), so the reference's load semantics are unchanged.
GPU_HBM_ACTIVITY_METRIC = "gpu_hbm_activity_avg"
# Measured on the MI355X calibration box (tools/hbm_share_calibration.py,
# profiles/gpu_calibration.md): amdgpu's mem_busy_percent averaged over 8 s of one tenant alone
# on the GPU. A streaming HBM copy reads 10.9 / 30.1 / 48.8 / 54.4 % holding 12.5 / 25 / 50 / 100 %
# of the CUs; a bf16 MFMA burn reads 0 % at 25, 75 and 100 %. Other boxes read the same kernels at
# the same GB/s on another scale (20.7 / 28.7 % for 25 / 100 % on one): the poller maps every
# reading onto this box's scale through the device's own calibration (GpuSpec.hbm_busy_cal,
# telemetry.store.normalize_hbm_activity) before these constants apply. The device mark fires
# for a streamer of a quarter of the GPU or more (30.1 on this scale): 0.20 leaves a single
# reading a third of margin under that mean, and stays over an eighth-GPU streamer (10.9).
HBM_HOT_THRESHOLD = 0.20
# (share %, mem_busy %) of a lone streaming tenant, from the same calibration: the learner's
# threshold for a pod alone on a device is HBM_LEARN_FRACTION of the curve at that pod's share
# (capped at the device threshold), so a lone 25 % streamer (30 %) is learned while a lone MFMA
# tenant of any size (0 %) is not.
HBM_STREAMING_CURVE = ((12.5, 10.9), (25.0, 30.1), (50.0, 48.8), (100.0, 54.4))
HBM_LEARN_FRACTION = 0.5
AMD_GPU_NODE_LABEL = ("amd.com/gpu.present", "true")   # default telemetry node selector

MI355X_CUS = 256
MI355X_XCDS = 8
MI355X_HBM_BYTES = 288 * 1000 ** 3   # datasheet; the agent reads the real value

DEFAULT_PORT = 39999                 # cmd/main.go:96-99
DEFAULT_POLICY_PATH = "/data/policy.yaml"          # cmd/main.go:34
DEFAULT_PROMETHEUS_URL = "http://thanos-prometheus.kube-system:80"  # cmd/main.go:66-67
FILTER_NODE_CACHE_ERROR = ("nano-gpu-scheduler extender must be configured with "
                           "nodeCacheCapable=true")   # routes.go:66


def container_annotation(name: str) -> str:
    return ANNOTATION_CONTAINER_FMT.format(name)

# the pod informer's field selector: assigned pods only (kube-scheduler's own assigned-pod
# informer uses the same selector)
ASSIGNED_PODS = "spec.nodeName!="
