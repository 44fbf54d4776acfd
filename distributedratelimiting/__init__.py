"""Import shim: ``distributedratelimiting.redis_amd`` is the package directory
``distributedratelimiting.redis_amd/`` at the repository root (linked as
``distributedratelimiting/redis_amd``)."""
