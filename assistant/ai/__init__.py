"""AI abstraction layer: providers (chat) and embedders, prefix-routed factories, dialog helper."""
