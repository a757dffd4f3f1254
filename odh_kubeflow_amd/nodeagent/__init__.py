"""Production node-side component: amdgpu telemetry and pod→GPU attribution (read-only)."""
