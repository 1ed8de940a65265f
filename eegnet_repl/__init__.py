"""Import-path shim: ``eegnet_repl.model`` resolves to the MI355X build (eegnetreplication_amd),
so code and tests written against PraKesEy/EEGNetReplication's package name run unchanged."""
