"""sentinel_amd -- MI355X-native batched token-decision engine for Sentinel's sliding-window
flow-control hot path (LeapArray/ClusterMetric + ClusterFlowChecker/ClusterParamFlowChecker behind
the TokenService SPI).  See DESIGN.md."""
from ._lib import SentinelError, load as load_library  # noqa: F401
from .token_service import (ClusterFlowConfig, ClusterRuleConstant, FlowRule, GpuTokenCluster,  # noqa: F401
                            GpuTokenService, LocalParamRule, ParamFlowRule, ServerNamespace, TokenResult,
                            TokenResultStatus)

__all__ = ["GpuTokenService", "GpuTokenCluster", "FlowRule", "ParamFlowRule", "LocalParamRule", "ClusterFlowConfig", "ClusterRuleConstant",
           "ServerNamespace", "TokenResult", "TokenResultStatus", "SentinelError", "load_library"]
