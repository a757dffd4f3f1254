"""Test-platform processes: dev apiserver, scheduler, fake kubelet."""
