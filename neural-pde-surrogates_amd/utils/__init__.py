from .attr import getattr_nested, rgetattr, rsetattr  # noqa: F401
