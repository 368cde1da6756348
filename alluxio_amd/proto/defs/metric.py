"""Metrics master service (package alluxio.grpc.metric).

Contract source: core/transport/src/main/proto/grpc/metric_master.proto:1-61.
"""

SCHEMA = r"""
package alluxio.grpc.metric
msg ClearMetricsPRequest
msg ClearMetricsPResponse
msg ClientMetrics source=1:str metrics=2:alluxio.grpc.Metric*
msg MetricsHeartbeatPOptions clientMetrics=1:ClientMetrics*
msg MetricsHeartbeatPRequest options=1:MetricsHeartbeatPOptions
msg MetricsHeartbeatPResponse
msg MetricValue doubleValue=1:f64 stringValue=2:str metricType=6:alluxio.grpc.MetricType
msg GetMetricsPOptions
msg GetMetricsPResponse metrics=1:{str,MetricValue}
rpc MetricsMasterClientService ClearMetrics ClearMetricsPRequest ClearMetricsPResponse
rpc MetricsMasterClientService MetricsHeartbeat MetricsHeartbeatPRequest MetricsHeartbeatPResponse
rpc MetricsMasterClientService GetMetrics GetMetricsPOptions GetMetricsPResponse
"""
