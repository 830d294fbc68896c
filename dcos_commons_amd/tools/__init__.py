"""Packaging and release tooling (reference: ``tools/``).

* ``universe``: package identity, universe repositories and the stub-universe builder;
* ``build_package``: build a framework's artifacts + stub universe, optionally publish it;
* ``publish_http`` / ``publish_dcos_file``: serve a build over HTTP / bundle it into a ``.dcos`` file;
* ``release_builder``: re-home a stub universe as a versioned release in a universe repository;
* ``airgap_linter``: reject packages that reach outside an air-gapped cluster;
* ``standardize_config_json``: canonical option order in ``config.json``.

Cloud uploaders (S3/Azure), Jenkins glue and the Go CLI build scripts of the reference have no
counterpart: there is no network here and the CLI is the native ``sdk-cli``.
"""
