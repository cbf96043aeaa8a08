from .app import create_app, KubectlService  # noqa: F401
